// Wide skinny GEMM for decode-shaped problems (M <= 64 activation rows), "skinny2":
//
//   C[m, n] = act(alpha * rstd[m] * sum_k X[m, k] * W[n, k] + bias[n]) (+ res_alpha * R[m, n]),  GLU optional
//
// Decode is weight-bandwidth bound; what limits the first skinny kernel (gemv.hip) at M = 64 is the LDS-DMA
// traffic per weight byte: its 64-row W tile streams together with a 64-row X tile (X : W bytes = M : BN
// = 1 : 1), so half of every CU's DMA issue and LDS writes carry activations that are the same for every
// workgroup, and its four waves split each K-step (cross-wave reduction at the end).  Here:
//
// * Workgroup = 4 waves, tile = 128 W rows (wave w owns rows [32 w, 32 w + 32)) x all M rows; every wave
//   consumes the WHOLE 64-wide K-step of its own rows -- 4 k16 slices x 2 X groups = 8 v_mfma_f32_32x32x16_bf16
//   per step, no cross-wave reduction: each wave's accumulators are its final (or split-K partial) outputs.
// * Per step: W tile 128 x 64 (16 KB) + X tile 64 x 64 (8 KB) by LDS-DMA (buffer_load ... lds, 16 B per
//   lane, range-checked zero fill for rows >= N / M and K tails), X : W = 1 : 2.  A ring of S2_STAGES
//   = 3 x 24 KB, so two workgroups fit a CU (four stages of W in flight per CU), or 6 x 24 KB for one; counted vmcnt + one
//   s_barrier per step.  The weight stream carries the nt cache policy (read once per decode step).
// * Folded RMSNorm (GemmArgs::rms): every wave accumulates the sum of squares of the X fragments it reads
//   anyway (the same for all waves: no sharing needed), rstd[m] is applied before the epilogue.
// * Split-K over kg workgroups per tile: fp32 partial slabs written through (sc1), an arrival ticket per tile
//   from this launch's ticket slice (skinny_ticket_slice), the last arriver sums the kg slabs in K-group
//   order with sc1 loads (the write-through hand-off of gemv.hip) and runs the fused epilogue.
#include "common.h"
#include "launchers.h"

namespace shai {

typedef __bf16 bf16x8w __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void s2_lds_void;

constexpr int S2_BN = 128;                     // W rows per workgroup
constexpr int S2_BK = 64;                      // K per step
constexpr int S2_MB = 64;                      // X rows (two 32-row groups)
constexpr int S2_W_ELEMS = S2_BN * S2_BK;      // 8192 bf16 = 16 KB
constexpr int S2_X_ELEMS = S2_MB * S2_BK;      // 4096 bf16 = 8 KB
constexpr int S2_STAGE = S2_W_ELEMS + S2_X_ELEMS;
constexpr int S2_PER = 6;                      // DMA wave-instructions per wave per step (4 W + 2 X)
constexpr uint32_t S2_OOB = 0x80000000u;
// ring depth: 3 stages (72 KB, two workgroups per CU) or 6 stages (144 KB, one workgroup per CU with five
// steps of W in flight -- for grids of about one tile per CU, e.g. lm_head / gate_up without split-K)
constexpr size_t s2_lds(int stages) { return (size_t)stages * S2_STAGE * 2; }

__device__ __forceinline__ int s2_swz(int row, int ch) { return row * S2_BK + ((ch ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t s2_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void s2_store_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)off, 0, 16);  // sc1: write-through
}
__device__ __forceinline__ float s2_load_wt(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 16));
}
typedef unsigned s2_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void s2_store4_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, const float* v) {
  s2_u4 u = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
  __builtin_amdgcn_raw_buffer_store_b128(u, r, (int)off, 0, 16);
}
__device__ __forceinline__ void s2_load4_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, float* v) {
  const s2_u4 u = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = __uint_as_float(u[i]);
}

template <int N>
__device__ __forceinline__ void s2_wait_upto(int pending) {
  if constexpr (N == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (pending >= N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N * S2_PER) : "memory");
    else s2_wait_upto<N - 1>(pending);
  }
}

// One output element pair / element: bias, activation (GLU: value * act(gate)), residual, bf16 store.
template <bool GLU, int ACT>
__device__ __forceinline__ void s2_store(const GemmArgs& p, int n, int m, float v0, float v1) {
  if (n >= p.N || m >= p.M) return;
  if constexpr (GLU) {
    const float a = v0 * p.alpha + (p.bias ? bf2f(p.bias[n]) : 0.f);
    const float g = v1 * p.alpha + (p.bias ? bf2f(p.bias[n + 1]) : 0.f);
    float o = a * apply_act<ACT>(g);
    const int nc = n >> 1;
    if (p.residual) o += bf2f(p.residual[(long)m * p.ldr + nc]) * p.res_alpha;
    p.C[(long)m * p.ldc + nc] = f2bf(o);
  } else {
    float o = apply_act<ACT>(v0 * p.alpha + (p.bias ? bf2f(p.bias[n]) : 0.f));
    if (p.residual) o += bf2f(p.residual[(long)m * p.ldr + n]) * p.res_alpha;
    p.C[(long)m * p.ldc + n] = f2bf(o);
  }
}

// Accumulator layout of v_mfma_f32_32x32x16 with W rows as A and X rows as B: lane (fr = lane & 31,
// fh = lane >> 5) holds D[n][m] for m = 32 j + fr and n = (r & 3) + 8 (r >> 2) + 4 fh, r = 0..15.
template <bool GLU, int ACT>
__device__ __forceinline__ void s2_epilogue(const GemmArgs& p, int nbase, int fr, int fh, const float (&v)[2][16],
                                            const float (&rs)[2]) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = 32 * j + fr;
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const int n = nbase + (r & 3) + 8 * (r >> 2) + 4 * fh;
      if constexpr (GLU) {
        s2_store<true, ACT>(p, n, m, v[j][r] * rs[j], v[j][r + 1] * rs[j]);
      } else {
        s2_store<false, ACT>(p, n, m, v[j][r] * rs[j], 0.f);
        s2_store<false, ACT>(p, n + 1, m, v[j][r + 1] * rs[j], 0.f);
      }
    }
  }
}

template <bool GLU, int ACT, bool RMS, int S2_STAGES>
__global__ void __launch_bounds__(256) skinny2_kernel(const GemmArgs p, float* __restrict__ ws, int kg_steps,
                                                      unsigned* __restrict__ cnt) {
  extern __shared__ __attribute__((aligned(16))) bf16_t s2_smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tile = blockIdx.x, kg = blockIdx.y, KG = gridDim.y;
  const int n0 = tile * S2_BN;
  const int ksteps = (p.K + S2_BK - 1) / S2_BK;
  const int t0 = kg * kg_steps;
  const int nk = max(0, min(ksteps, t0 + kg_steps) - t0);

  const __amdgpu_buffer_rsrc_t rW = s2_rsrc(p.W, (uint32_t)min((long)p.N * p.ldw * 2, 0x7fffffffL));
  const __amdgpu_buffer_rsrc_t rX = s2_rsrc(p.A, (uint32_t)min((long)p.M * p.lda * 2, 0x7fffffffL));

  // DMA geometry: a wave instruction fills 8 LDS rows x 128 B lane-linearly; the lane at chunk position
  // lpos fetches global chunk lpos ^ swz(row) (source-side swizzle, conflict-free ds_read_b128 later).
  const int lrow = lane >> 3, lpos = lane & 7;
  uint32_t woff[4], xoff[2];
  int wrow[4], xrow[2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    wrow[j] = (w * 4 + j) * 8 + lrow;          // W tile rows 32 w .. 32 w + 31
    const int n = n0 + wrow[j], ch = lpos ^ ((wrow[j] >> 1) & 7);
    woff[j] = n < p.N ? (uint32_t)(((long)n * p.ldw + ch * 8) * 2) : S2_OOB;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    xrow[j] = (w * 2 + j) * 8 + lrow;          // X rows 16 w .. 16 w + 15
    const int ch = lpos ^ ((xrow[j] >> 1) & 7);
    xoff[j] = xrow[j] < p.M ? (uint32_t)(((long)xrow[j] * p.lda + ch * 8) * 2) : S2_OOB;
  }
  auto stage = [&](int buf, int step) {
    bf16_t* sw = s2_smem + buf * S2_STAGE;
    bf16_t* sx = sw + S2_W_ELEMS;
    const int k0 = (t0 + step) * S2_BK;
    const bool kin = k0 < p.K;  // K tail: whole chunks past K read as zeros (K % 8 == 0)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ch = lpos ^ ((wrow[j] >> 1) & 7);
      const uint32_t off = (woff[j] != S2_OOB && kin && k0 + ch * 8 < p.K) ? woff[j] + (uint32_t)(k0 * 2) : S2_OOB;
      if (p.w_nt) __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (s2_lds_void*)(sw + (w * 4 + j) * 8 * S2_BK), 16, off, 0, 0, 2);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (s2_lds_void*)(sw + (w * 4 + j) * 8 * S2_BK), 16, off, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ch = lpos ^ ((xrow[j] >> 1) & 7);
      const uint32_t off = (xoff[j] != S2_OOB && kin && k0 + ch * 8 < p.K) ? xoff[j] + (uint32_t)(k0 * 2) : S2_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (s2_lds_void*)(sx + (w * 2 + j) * 8 * S2_BK), 16, off, 0, 0, 0);
    }
  };

  float16_ acc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
  float ss[2] = {0.f, 0.f};  // folded RMSNorm: this lane's share of sum_k X[m, k]^2 (m = 32 j + fr)
  const int fr = lane & 31, fh = lane >> 5;
#pragma unroll
  for (int i = 0; i < S2_STAGES - 1; ++i)
    if (i < nk) stage(i, i);
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    s2_wait_upto<S2_STAGES - 2>(min(S2_STAGES - 2, nk - 1 - kt));
    __builtin_amdgcn_s_barrier();
    if (kt + S2_STAGES - 1 < nk) {
      const int nb = buf == 0 ? S2_STAGES - 1 : buf - 1;  // buffer of step kt-1: every wave is past it
      stage(nb, kt + S2_STAGES - 1);
    }
    const bf16_t* sw = s2_smem + buf * S2_STAGE;
    const bf16_t* sx = sw + S2_W_ELEMS;
#pragma unroll
    for (int s = 0; s < 4; ++s) {  // k16 slices of the step
      const int ch = 2 * s + fh;
      const bf16x8w wf = *reinterpret_cast<const bf16x8w*>(sw + s2_swz(32 * w + fr, ch));
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16x8w xf = *reinterpret_cast<const bf16x8w*>(sx + s2_swz(32 * j + fr, ch));
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf, xf, acc[j], 0, 0, 0);
        if constexpr (RMS) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float f = (float)xf[e];
            ss[j] = fmaf(f, f, ss[j]);
          }
        }
      }
    }
    buf = buf == S2_STAGES - 1 ? 0 : buf + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (RMS) {  // both K halves of row m: lanes fr and fr + 32
#pragma unroll
    for (int j = 0; j < 2; ++j) ss[j] += __shfl_xor(ss[j], 32, 64);
  }
  float v[2][16];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) v[j][r] = acc[j][r];
  const int nbase = n0 + 32 * w;
  if (KG == 1) {
    float rs[2] = {1.f, 1.f};
    if constexpr (RMS) {
#pragma unroll
      for (int j = 0; j < 2; ++j) rs[j] = rsqrtf(ss[j] / p.K + p.rms_eps);
    }
    s2_epilogue<GLU, ACT>(p, nbase, fr, fh, v, rs);
    return;
  }
  // ---- split-K: slab [tile][kg] = 8 chunks of 256 lanes x 4 floats (chunk c = 4 consecutive accumulator
  // registers of one X group: coalesced 16-byte stores / loads, 4 KB per wave instruction) + 64 row sums of
  // squares.  The write-through publish form (every wave drains, barrier, one relaxed agent-scope ticket; the
  // last arriver reads only sc1 loads into registers).
  constexpr int SLAB = 8 * 256 * 4 + S2_MB;
  const __amdgpu_buffer_rsrc_t rws = s2_rsrc(ws, 0x7fffffffu);
  const uint32_t tile_base = (uint32_t)((long)tile * KG * SLAB * 4);
  const uint32_t my_base = tile_base + (uint32_t)(kg * SLAB * 4);
  auto chunk_off = [&](int c) { return (uint32_t)((c * 256 + tid) * 16); };
#pragma unroll
  for (int c = 0; c < 8; ++c) s2_store4_wt(rws, my_base + chunk_off(c), &v[c >> 2][(c & 3) * 4]);
  if constexpr (RMS) {
    if (w == 0 && fh == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j) s2_store_wt(rws, my_base + (uint32_t)((8 * 256 * 4 + 32 * j + fr) * 4), ss[j]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ unsigned s2_last;
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(&cnt[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    s2_last = old == (unsigned)(KG - 1);
  }
  __syncthreads();
  if (s2_last == 0u) return;
  if (tid == 0) __hip_atomic_store(&cnt[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // sum the KG slabs in K-group order (own slab from registers; two slabs' loads in flight before their
  // adds): the result does not depend on arrival order
  float sum[2][16], ssum[2] = {0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) sum[j][r] = 0.f;
  for (int q0 = 0; q0 < KG; q0 += 2) {
    float t[2][2][16], ts[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = q0 + u < KG ? q0 + u : kg;  // past KG / own slot: re-read own slab, dropped below
      const uint32_t b = tile_base + (uint32_t)(q * SLAB * 4);
#pragma unroll
      for (int c = 0; c < 8; ++c) s2_load4_wt(rws, b + chunk_off(c), &t[u][c >> 2][(c & 3) * 4]);
      if constexpr (RMS) {
#pragma unroll
        for (int j = 0; j < 2; ++j) ts[u][j] = s2_load_wt(rws, b + (uint32_t)((8 * 256 * 4 + 32 * j + fr) * 4));
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = q0 + u;
      if (q >= KG) continue;
      const bool mine = q == kg;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sum[j][r] += mine ? v[j][r] : t[u][j][r];
        if constexpr (RMS) ssum[j] += mine ? ss[j] : ts[u][j];
      }
    }
  }
  float rs[2] = {1.f, 1.f};
  if constexpr (RMS) {
#pragma unroll
    for (int j = 0; j < 2; ++j) rs[j] = rsqrtf(ssum[j] / p.K + p.rms_eps);
  }
  s2_epilogue<GLU, ACT>(p, nbase, fr, fh, sum, rs);
}

bool skinny2_supported(const GemmArgs& a) {
  // (QUICK_GELU is not instantiated by launch_skinny2: such problems stay on the other kernels)
  return a.M >= 1 && a.M <= S2_MB && !a.conv && a.batch <= 1 && a.w_slice_rows == 0 && a.w_scale == nullptr &&
         a.bias2d == nullptr &&
         a.act != ACT_QUICK_GELU &&
         a.gate == nullptr && a.row_mr == nullptr && a.K % 8 == 0 && a.lda % 8 == 0 && a.ldw % 8 == 0 && (!a.glu || a.N % 2 == 0) &&
         (long)a.N * a.ldw * 2 < 0x7fffffffL && (long)a.M * a.lda * 2 < 0x7fffffffL;
}

int skinny2_max_kgroups(const GemmArgs& a) {
  const int ksteps = (a.K + S2_BK - 1) / S2_BK;
  int kg = 1;
  while (kg < 16 && ksteps / (kg * 2) >= 2) kg *= 2;
  return kg;
}

size_t skinny2_workspace_bytes(const GemmArgs& a, int kg) {
  if (kg <= 1) return 0;
  const size_t tiles = (a.N + S2_BN - 1) / S2_BN;
  return tiles * kg * (size_t)(8 * 256 * 4 + S2_MB) * sizeof(float);
}

// kg > 1 needs ws (skinny2_workspace_bytes) and a ticket slice; without either it runs with kg = 1.
void launch_skinny2(const GemmArgs& a_in, float* ws, int kg, bool deep, hipStream_t s) {
  static const int nt = [] {
    const char* e = getenv("SHAI_SKINNY_NT");
    return e ? atoi(e) : 1;
  }();
  GemmArgs a = a_in;
  a.w_nt = nt;
  const int ksteps = (a.K + S2_BK - 1) / S2_BK;
  const int tiles = (a.N + S2_BN - 1) / S2_BN;
  if (kg > ksteps) kg = ksteps;
  unsigned* cnt = nullptr;
  if (kg > 1 && ws != nullptr) cnt = skinny_ticket_slice(s, tiles);
  if (cnt == nullptr) kg = 1;
  const int kg_steps = (ksteps + kg - 1) / kg;
  kg = (ksteps + kg_steps - 1) / kg_steps;  // no empty K groups (their tickets would never arrive)
  dim3 grid(tiles, kg), block(256);
#define S2R(G, A, ST)                                                                                   \
  do {                                                                                                  \
    if (a.rms) skinny2_kernel<G, A, true, ST><<<grid, block, s2_lds(ST), s>>>(a, ws, kg_steps, cnt);    \
    else skinny2_kernel<G, A, false, ST><<<grid, block, s2_lds(ST), s>>>(a, ws, kg_steps, cnt);         \
  } while (0)
#define S2(G, A)              \
  do {                        \
    if (deep) S2R(G, A, 6);   \
    else S2R(G, A, 3);        \
  } while (0)
#define S2_ACT(G)                                      \
  switch (a.act) {                                     \
    case ACT_SILU: S2(G, ACT_SILU); break;             \
    case ACT_GELU: S2(G, ACT_GELU); break;             \
    case ACT_GELU_TANH: S2(G, ACT_GELU_TANH); break;   \
    case ACT_RELU: S2(G, ACT_RELU); break;             \
    default: S2(G, ACT_NONE); break;                   \
  }
  if (a.glu) {
    S2_ACT(true)
  } else {
    S2_ACT(false)
  }
#undef S2_ACT
#undef S2
#undef S2R
}

}  // namespace shai
