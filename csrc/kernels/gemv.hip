// Skinny GEMM for decode-shaped problems (M <= 32 activation rows, e.g. LLM
// decode batches, Flux/SD modulation GEMMs with few rows):
//
//   C[m, n] = act(alpha * sum_k X[m, k] * W[n, k] + bias[n]) (+ res_alpha * R[m, n]),  GLU optional
//
// The problem is purely weight-bandwidth bound (W is read once, X is tiny and
// L2-resident), so the kernel is organised around streaming W at HBM rate:
//
// * A workgroup owns 32 output columns n (= 32 rows of W) and a K range; its 8
//   waves split that range.  Each wave runs 32x32x16 bf16 MFMAs with W as the A
//   operand (rows n) and X^T as B (columns m; rows m >= M read as zero).
// * K permutation: a lane (row r = lane & 31, half h = lane >> 5) loads 64
//   contiguous bytes of its W row per 64-wide K step (4 x dwordx4, nontemporal
//   so W does not evict X from L2) and feeds them to 4 MFMAs; X fragments use
//   the same permuted K order, so the dot products are unchanged.  The next K
//   step's loads are issued before the current step's MFMAs (register double
//   buffer).
// * Cross-wave reduction through LDS (padded, conflict-free), then either the
//   fused epilogue directly (one K group) or, when more parallelism is needed
//   to fill 256 CUs, a split over KG workgroups: each writes its fp32 partial
//   tile, and the LAST workgroup to arrive (atomic ticket per tile; it resets
//   the ticket, so the kernel is HIP-graph replay safe) sums the partials and
//   runs the epilogue -- one launch, no separate reduce kernel.
#include "common.h"
#include "launchers.h"

namespace shai {

typedef __bf16 bf16x8s __attribute__((ext_vector_type(8)));

constexpr int SK_WAVES = 8;
constexpr int SK_PAD = 33;

template <bool GLU, int ACT>
__device__ __forceinline__ void skinny_store(const GemmArgs& p, int n0, int m, int nl, float v0, float v1) {
  // v0 = value at column n0 + nl, v1 = value at n0 + nl + 1 (used by GLU only)
  const int n = n0 + nl;
  if constexpr (GLU) {
    if (n >= p.N) return;
    const float a = v0 * p.alpha + (p.bias ? bf2f(p.bias[n]) : 0.f);
    const float g = v1 * p.alpha + (p.bias ? bf2f(p.bias[n + 1]) : 0.f);
    float o = a * apply_act<ACT>(g);
    const int nc = n >> 1;
    if (p.residual) o += bf2f(p.residual[(long)m * p.ldr + nc]) * p.res_alpha;
    p.C[(long)m * p.ldc + nc] = f2bf(o);
  } else {
    if (n >= p.N) return;
    float o = apply_act<ACT>(v0 * p.alpha + (p.bias ? bf2f(p.bias[n]) : 0.f));
    if (p.residual) o += bf2f(p.residual[(long)m * p.ldr + n]) * p.res_alpha;
    p.C[(long)m * p.ldc + n] = f2bf(o);
  }
}

template <bool GLU, int ACT>
__global__ void __launch_bounds__(SK_WAVES * 64) skinny_gemm_kernel(const GemmArgs p, float* __restrict__ ws,
                                                                    int* __restrict__ tickets, int kg_steps) {
  __shared__ float red[SK_WAVES][32][SK_PAD];
  __shared__ int last;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile = blockIdx.x;
  const int kg = blockIdx.y, KG = gridDim.y;
  const int n0 = tile * 32;
  const int r = lane & 31, h = lane >> 5;

  // K steps (64 wide) of this workgroup, split over the waves
  const int ksteps = p.K >> 6;
  const int g0 = kg * kg_steps, g1 = min(ksteps, g0 + kg_steps);
  const int per = (g1 - g0 + SK_WAVES - 1) / SK_WAVES;
  const int s0 = g0 + w * per, s1 = min(g1, s0 + per);

  const bf16_t* wrow = p.W + (long)min(n0 + r, p.N - 1) * p.ldw + 32 * h;
  // rows m >= M re-read row M-1: they only feed output columns m >= M, which are never stored
  const bf16_t* xrow = p.A + (long)min(r, p.M - 1) * p.lda + 32 * h;
  float16_ acc = {};

  // Batched issue: all loads of U consecutive K steps go out back to back (U x 8
  // dwordx4 per lane, 32 KB per wave in flight), then their MFMAs run.  Other
  // waves' loads overlap this wave's (short) MFMA phase.  A software-pipelined
  // ping-pong variant was defeated by the compiler's register reuse.
  constexpr int U = 4;
  for (int s = s0; s < s1; s += U) {
    uint4_ wv[U][4], xv[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (s + u < s1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          wv[u][j] = __builtin_nontemporal_load(reinterpret_cast<const uint4_*>(wrow + ((s + u) << 6) + 8 * j));
          xv[u][j] = *reinterpret_cast<const uint4_*>(xrow + ((s + u) << 6) + 8 * j);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (s + u < s1) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8s, wv[u][j]),
                                                         __builtin_bit_cast(bf16x8s, xv[u][j]), acc, 0, 0, 0);
      }
    }
  }
  // C layout: lane column m = lane & 31; rows nl = (i & 3) + 8 * (i >> 2) + 4 * h
#pragma unroll
  for (int i = 0; i < 16; ++i) red[w][(i & 3) + 8 * (i >> 2) + 4 * h][r] = acc[i];
  __syncthreads();

  const int tid = threadIdx.x;
  if (KG == 1) {
    if constexpr (GLU) {
      const int m = tid >> 4, nl = (tid & 15) * 2;  // 512 threads = 32 m x 16 pairs
      if (m < p.M) {
        float v0 = 0.f, v1 = 0.f;
#pragma unroll
        for (int q = 0; q < SK_WAVES; ++q) {
          v0 += red[q][nl][m];
          v1 += red[q][nl + 1][m];
        }
        skinny_store<GLU, ACT>(p, n0, m, nl, v0, v1);
      }
    } else {
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int idx = tid + it * 512;
        const int m = idx >> 5, nl = idx & 31;
        if (m < p.M) {
          float v = 0.f;
#pragma unroll
          for (int q = 0; q < SK_WAVES; ++q) v += red[q][nl][m];
          skinny_store<GLU, ACT>(p, n0, m, nl, v, 0.f);
        }
      }
    }
    return;
  }

  // ---- split over KG workgroups: write this group's partial, last arrival reduces
  float* part = ws + ((long)kg * gridDim.x + tile) * 1024;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = tid + it * 512;
    const int m = idx >> 5, nl = idx & 31;
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < SK_WAVES; ++q) v += red[q][nl][m];
    part[idx] = v;
  }
  __threadfence();
  __syncthreads();
  if (tid == 0) {
    const int t = atomicAdd(&tickets[tile], 1);
    last = (t == KG - 1);
    if (last) tickets[tile] = 0;  // re-arm for the next launch / graph replay
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  if constexpr (GLU) {
    const int m = tid >> 4, nl = (tid & 15) * 2;
    if (m < p.M) {
      float v0 = 0.f, v1 = 0.f;
      for (int q = 0; q < KG; ++q) {
        const float* pp = ws + ((long)q * gridDim.x + tile) * 1024 + m * 32 + nl;
        v0 += __builtin_nontemporal_load(pp);
        v1 += __builtin_nontemporal_load(pp + 1);
      }
      skinny_store<GLU, ACT>(p, n0, m, nl, v0, v1);
    }
  } else {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int idx = tid + it * 512;
      const int m = idx >> 5, nl = idx & 31;
      if (m < p.M) {
        float v = 0.f;
        for (int q = 0; q < KG; ++q) v += __builtin_nontemporal_load(ws + ((long)q * gridDim.x + tile) * 1024 + idx);
        skinny_store<GLU, ACT>(p, n0, m, nl, v, 0.f);
      }
    }
  }
}

// ---------------------------------------------------------------------------- host side
bool skinny_supported(const GemmArgs& a) {
  return !a.conv && (a.batch <= 1) && a.M >= 1 && a.M <= 32 && a.K % 64 == 0 && a.N % 32 == 0 &&
         a.bias2d == nullptr && a.gate == nullptr && a.in_scale == nullptr && (a.lda % 8) == 0 && (a.ldw % 8) == 0;
}

// Number of K groups: enough workgroups to cover the CUs twice, each wave >= 2 K steps.
int skinny_kgroups(const GemmArgs& a) {
  const int tiles = a.N / 32, ksteps = a.K / 64;
  int kg = 1;
  while (tiles * kg < 512 && ksteps / (kg * 2) >= 2 * SK_WAVES) kg *= 2;
  return kg;
}

size_t skinny_workspace_bytes(const GemmArgs& a) {
  const int kg = skinny_kgroups(a);
  return kg > 1 ? (size_t)kg * (a.N / 32) * 1024 * sizeof(float) : 0;
}

void launch_skinny(const GemmArgs& a, float* ws, int* tickets, hipStream_t s) {
  const int kg = (ws != nullptr && tickets != nullptr) ? skinny_kgroups(a) : 1;
  const int ksteps = a.K / 64;
  const int kg_steps = (ksteps + kg - 1) / kg;
  dim3 grid(a.N / 32, kg), block(SK_WAVES * 64);
#define SK(G, A) skinny_gemm_kernel<G, A><<<grid, block, 0, s>>>(a, ws, tickets, kg_steps)
#define SK_ACT(G)                                    \
  switch (a.act) {                                   \
    case ACT_SILU: SK(G, ACT_SILU); break;           \
    case ACT_GELU: SK(G, ACT_GELU); break;           \
    case ACT_GELU_TANH: SK(G, ACT_GELU_TANH); break; \
    case ACT_QUICK_GELU: SK(G, ACT_QUICK_GELU); break; \
    case ACT_RELU: SK(G, ACT_RELU); break;           \
    default: SK(G, ACT_NONE); break;                 \
  }
  if (a.glu) {
    SK_ACT(true)
  } else {
    SK_ACT(false)
  }
#undef SK_ACT
#undef SK
}

}  // namespace shai
