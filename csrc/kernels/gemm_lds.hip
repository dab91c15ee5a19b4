// bf16 MFMA GEMM / implicit-GEMM convolution, v2: LDS-DMA staging.
//
//   C[b,m,n] = gate[(b*M+m)/G, n] * act(alpha * sum_k A[b,m,k] * W[b,n,k] + bias[n] + bias2d[m/R, n])
//              + res_alpha * Res[b,m,n]
//
// (gate: optional AdaLN-Zero gate rows, e.g. Flux gate_msa / gate_mlp per image.)
//
// Operand tiles move global -> LDS with `buffer_load_dwordx4 ... lds` (no VGPR
// round trip, no ds_write).  The buffer descriptor's range check supplies the
// zero fill: out-of-range lanes (M/N/K tails, conv padding taps) point past
// num_records and read 0, so the implicit-GEMM conv gather needs no branches
// around its loads.  The LDS image is lane-linear per wave instruction (8 rows x
// 128 B), so the XOR bank swizzle is applied to the per-lane SOURCE chunk and
// the same XOR on the ds_read_b128 side (guide rule 21).
//
// Tile configs (BM x BN, waves WM x WN, each wave 64 x (BN/WN) of 32x32 MFMA
// blocks), BK = 64, 2 LDS stages, loads for K-tile t+1 issued before the MFMAs
// of tile t, one vmcnt(0)+barrier per K-tile.  Optional split-K writes fp32
// partials that gemm_splitk_reduce folds together with the full epilogue.
// XCD-aware bijective block remap + grouped ordering along M.
#include "common.h"
#include "launchers.h"
#include "gemm_epilogue.h"

#include <algorithm>
#include <cstdlib>

namespace shai {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BK2 = 64;
constexpr uint32_t OOB = 0x80000000u;

__device__ __forceinline__ int swz2(int row, int ch) { return row * BK2 + ((ch ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, bf16_t* lds_wave_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds_wave_base, 16, voff, 0, 0, 0);
}

template <int BM, int BN, int WM, int WN, bool CONV, bool FAST, bool GLU, int ACT, bool SPLITK, int STAGES>
__global__ void __launch_bounds__(WM * WN * 64) gemm2_kernel(const GemmArgs p, float* __restrict__ ws, int k_per_split,
                                                             unsigned* __restrict__ cnt) {
  constexpr int NW = WM * WN;
  constexpr int NT = NW * 64;
  constexpr int TM = BM / WM, TN = BN / WN;     // wave tile
  constexpr int IM = TM / 32, JN = TN / 32;     // 32x32 blocks per wave
  constexpr int JA = BM / 8 / NW;               // A wave-instructions per K tile
  constexpr int JB = BN / 8 / NW;               // W wave-instructions per K tile
  static_assert(JA >= 1 && JB >= 1 && IM >= 1 && JN >= 1, "bad tile config");
  constexpr int STAGE = (BM + BN) * BK2;        // elements per stage
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;

  // ---- tile mapping (XCD remap + grouped M ordering)
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int total = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = total >> 3, r = total & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  constexpr int GROUP = 8;
  const int group = bid / (GROUP * tiles_n);
  const int first_m = group * GROUP;
  const int gsize = min(tiles_m - first_m, GROUP);
  const int in_group = bid - group * GROUP * tiles_n;
  const int m0 = (first_m + in_group % gsize) * BM;
  const int n0 = (in_group / gsize) * BN;
  const int b = SPLITK ? 0 : blockIdx.y;
  const int kz = SPLITK ? blockIdx.y : 0;
  const int k_begin = kz * k_per_split;
  const int k_end = min(p.K, k_begin + k_per_split);

  const bf16_t* A = p.A + (long)b * p.batch_a;
  const bf16_t* Wt = p.W + (long)b * p.batch_w;

  // ---- buffer descriptors (range check = zero fill)
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(Wt, (uint32_t)min((long)p.N * p.ldw * 2, 0x7fffffffL));
  __amdgpu_buffer_rsrc_t rA, rA2;
  if constexpr (CONV) {
    rA = make_rsrc(A, (uint32_t)min((long)p.Nimg * p.H * p.Wd * (p.A2 ? p.Cin1 : p.Cin) * 2, 0x7fffffffL));
    rA2 = p.A2 ? make_rsrc(p.A2, (uint32_t)min((long)p.Nimg * p.H * p.Wd * (p.Cin - p.Cin1) * 2, 0x7fffffffL))
               : rA;
  } else {
    rA = make_rsrc(A, (uint32_t)min((long)p.M * p.lda * 2, 0x7fffffffL));
    rA2 = rA;
  }

  // ---- per-lane staging geometry
  const int lrow = lane >> 3;      // row within an 8-row wave instruction
  const int lpos = lane & 7;       // LDS chunk position
  int a_row[JA], a_ch[JA];
  int cn[JA], coh[JA], cow[JA];
  bool cvalid[JA];
#pragma unroll
  for (int j = 0; j < JA; ++j) {
    const int r = (wid * JA + j) * 8 + lrow;
    a_row[j] = r;
    a_ch[j] = lpos ^ ((r >> 1) & 7);
    if constexpr (CONV) {
      const int m = m0 + r;
      cvalid[j] = m < p.M;
      const int mm = cvalid[j] ? m : 0;
      const int hw = p.OH * p.OW;
      cn[j] = mm / hw;
      const int rem = mm - cn[j] * hw;
      coh[j] = rem / p.OW;
      cow[j] = rem - coh[j] * p.OW;
    }
  }
  int w_row[JB], w_ch[JB];
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    const int r = (wid * JB + j) * 8 + lrow;
    w_row[j] = r;
    w_ch[j] = lpos ^ ((r >> 1) & 7);
  }

  auto stage = [&](int buf, int k0) {
    bf16_t* sa = smem + buf * STAGE;
    bf16_t* sw = sa + BM * BK2;
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const int n = n0 + w_row[j], k = k0 + w_ch[j] * 8;
      const uint32_t off = (n < p.N && k < k_end) ? (uint32_t)(((long)n * p.ldw + k) * 2) : OOB;
      glds16(rW, sw + (wid * JB + j) * 8 * BK2, off);
    }
    if constexpr (!CONV) {
#pragma unroll
      for (int j = 0; j < JA; ++j) {
        const int m = m0 + a_row[j], k = k0 + a_ch[j] * 8;
        const uint32_t off = (m < p.M && k < k_end) ? (uint32_t)(((long)m * p.lda + k) * 2) : OOB;
        glds16(rA, sa + (wid * JA + j) * 8 * BK2, off);
      }
    } else {
      int tapF = 0, c0F = 0;
      bool secondF = false;
      if constexpr (FAST) {
        tapF = k0 / p.Cin;
        c0F = k0 - tapF * p.Cin;
        secondF = p.A2 != nullptr && c0F >= p.Cin1;
      }
#pragma unroll
      for (int j = 0; j < JA; ++j) {
        const int k = k0 + a_ch[j] * 8;
        int tap, c;
        bool second;
        if constexpr (FAST) {
          tap = tapF;
          c = c0F + a_ch[j] * 8;
          second = secondF;
        } else {
          tap = k / p.Cin;
          c = k - tap * p.Cin;
          second = p.A2 != nullptr && c >= p.Cin1;
        }
        const int kh = tap / p.KW, kw = tap - kh * p.KW;
        int ih, iw;
        bool ok = cvalid[j] && k < k_end;
        if (p.upsample) {
          const int uh = coh[j] - p.pad + kh, uw = cow[j] - p.pad + kw;
          ok = ok && uh >= 0 && uh < 2 * p.H && uw >= 0 && uw < 2 * p.Wd;
          ih = uh >> 1;
          iw = uw >> 1;
        } else {
          ih = coh[j] * p.stride - p.pad + kh;
          iw = cow[j] * p.stride - p.pad + kw;
          ok = ok && ih >= 0 && ih < p.H && iw >= 0 && iw < p.Wd;
        }
        const int cs = p.A2 ? (second ? p.Cin - p.Cin1 : p.Cin1) : p.Cin;
        const int cc = second ? c - p.Cin1 : c;
        const uint32_t off = ok ? (uint32_t)(((((long)cn[j] * p.H + ih) * p.Wd + iw) * cs + cc) * 2) : OOB;
        if constexpr (FAST) {
          glds16(secondF ? rA2 : rA, sa + (wid * JA + j) * 8 * BK2, off);
        } else {
          // non-uniform source choice: two masked loads into the same LDS slot are not allowed,
          // so a per-lane selected descriptor is not expressible; the generic path needs A2 == null.
          glds16(rA, sa + (wid * JA + j) * 8 * BK2, off);
        }
      }
    }
  };

  float16_ acc[IM][JN];
#pragma unroll
  for (int i = 0; i < IM; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = k_end > k_begin ? (k_end - k_begin + BK2 - 1) / BK2 : 0;
  const int fr = lane & 31, fh = lane >> 5;
  auto compute = [&](int buf) {
    const bf16_t* sa = smem + buf * STAGE;
    const bf16_t* sw = sa + BM * BK2;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 af[IM], wf[JN];
#pragma unroll
      for (int i = 0; i < IM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(sa + swz2(wm * TM + i * 32 + fr, 2 * s + fh));
#pragma unroll
      for (int j = 0; j < JN; ++j) wf[j] = *reinterpret_cast<const bf16x8*>(sw + swz2(wn * TN + j * 32 + fr, 2 * s + fh));
#pragma unroll
      for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[j], af[i], acc[i][j], 0, 0, 0);
    }
  };

  if constexpr (STAGES == 2) {
    if (nk > 0) {
      stage(0, k_begin);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) stage(cur ^ 1, k_begin + (kt + 1) * BK2);
      compute(cur);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    // 3 LDS stages: tiles t+1 and t+2 stay in flight while tile t is consumed.
    // Per iteration: counted vmcnt retires this wave's DMA of tile t (FIFO), a raw
    // s_barrier makes every wave's part visible AND proves all waves finished reading
    // the buffer of tile t-1, which is then refilled with tile t+2.
    constexpr int PER = JA + JB;  // DMA instructions per wave per tile
    if (nk > 0) stage(0, k_begin);
    if (nk > 1) stage(1, k_begin + BK2);
    int buf = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + 2 < nk) stage(buf == 0 ? 2 : buf - 1, k_begin + (kt + 2) * BK2);
      compute(buf);
      buf = buf == 2 ? 0 : buf + 1;
    }
  }

  // ---- epilogue: lane owns row m, 4 groups of 4 consecutive n per 32x32 block
  // In-launch split-K fixup (tiles with <= 4 32x32 blocks per wave; the skinny kernel's write-through hand-off, gemv.hip): every K group
  // stores its fp32 partial tile write-through (sc1), drains, joins the barrier and takes a ticket; the group
  // drawing the last one re-arms it, sums the slabs in K-group order (its own from registers, so the sum matches
  // the separate fold bit for bit whatever the arrival order) and runs the full epilogue.  Batch-1 SD2.1 steps
  // run most of their GEMMs split-K at these tiles: the fold kernel was 8.7 % of their kernel time.
  constexpr bool FIXOK = IM * JN <= 4 && !(BM == 128 && BN == 128);
  if constexpr (SPLITK && FIXOK) {
    if (cnt != nullptr) {
      __shared__ unsigned g2_last;
      const int S = gridDim.y;
      const __amdgpu_buffer_rsrc_t rws = make_rsrc(ws, (uint32_t)min((long)S * p.M * p.N * 4, 0x7fffffffL));
#pragma unroll
      for (int i = 0; i < IM; ++i) {
        const int m = m0 + wm * TM + i * 32 + fr;
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int n = n0 + wn * TN + j * 32 + 8 * g + 4 * fh;
            const uint32_t off = (uint32_t)(((long)kz * p.M * p.N + (long)m * p.N + n) * 4);
            if (m < p.M && n + 3 < p.N) {
              const float4_ v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4_, v), rws, (int)off, 0, 16);
            } else if (m < p.M) {
              for (int e = 0; e < 4 && n + e < p.N; ++e)
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][4 * g + e]), rws, (int)(off + 4 * e), 0,
                                                      16);
            }
          }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const unsigned old = __hip_atomic_fetch_add(&cnt[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        g2_last = old == (unsigned)(S - 1);
      }
      __syncthreads();
      if (g2_last == 0u) return;
      if (tid == 0) __hip_atomic_store(&cnt[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // slabs in rounds of U: every (i, j, g) group's loads of the round are issued before the first add (a
      // load-add chain per slab and group made the fixup latency-bound); the own slab is re-read and replaced by
      // the registers, so the sum order is the K-group order
      float4_ tot[IM][JN][4];
#pragma unroll
      for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) tot[i][j][g] = float4_{0.f, 0.f, 0.f, 0.f};
      constexpr int U = IM * JN <= 2 ? 2 : 1;  // slabs per round (registers: U x the tile's accumulators)
      for (int q0 = 0; q0 < S; q0 += U) {
        float4_ ld[U][IM][JN][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int q = min(q0 + u, S - 1);
#pragma unroll
          for (int i = 0; i < IM; ++i) {
            const int m = min(m0 + wm * TM + i * 32 + fr, p.M - 1);
#pragma unroll
            for (int j = 0; j < JN; ++j)
#pragma unroll
              for (int g = 0; g < 4; ++g) {
                const int n = min(n0 + wn * TN + j * 32 + 8 * g + 4 * fh, ((p.N - 1) & ~3));
                const uint32_t off = (uint32_t)(((long)q * p.M * p.N + (long)m * p.N + n) * 4);
                ld[u][i][j][g] = __builtin_bit_cast(float4_, __builtin_amdgcn_raw_buffer_load_b128(rws, (int)off, 0, 16));
              }
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int q = q0 + u;
          if (q >= S) continue;
#pragma unroll
          for (int i = 0; i < IM; ++i)
#pragma unroll
            for (int j = 0; j < JN; ++j)
#pragma unroll
              for (int g = 0; g < 4; ++g) {
                const float4_ own = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
                tot[i][j][g] += q == kz ? own : ld[u][i][j][g];
              }
        }
      }
#pragma unroll
      for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[i][j][4 * g + e] = tot[i][j][g][e];
      bf16_t* C = p.C;
#pragma unroll
      for (int i = 0; i < IM; ++i) {
        const int m = m0 + wm * TM + i * 32 + fr;
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int n = n0 + wn * TN + j * 32 + 8 * g + 4 * fh;
            if (n >= p.N) continue;
            float v[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
            epilogue4<GLU, ACT>(p, C, p.residual, m, n, v, 0);
          }
      }
      return;
    }
  }
  if constexpr (SPLITK) {
    float* W = ws + (long)kz * p.M * p.N;
#pragma unroll
    for (int i = 0; i < IM; ++i) {
      const int m = m0 + wm * TM + i * 32 + fr;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < JN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = n0 + wn * TN + j * 32 + 8 * g + 4 * fh;
          if (n + 3 < p.N) {
            float4_ v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
            *reinterpret_cast<float4_*>(W + (long)m * p.N + n) = v;
          } else {
            for (int e = 0; e < 4 && n + e < p.N; ++e) W[(long)m * p.N + n + e] = acc[i][j][4 * g + e];
          }
        }
    }
  } else {
    bf16_t* C = p.C + (long)b * p.batch_c;
    const bf16_t* R = p.residual ? p.residual + (long)b * p.batch_r : nullptr;
#pragma unroll
    for (int i = 0; i < IM; ++i) {
      const int m = m0 + wm * TM + i * 32 + fr;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < JN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = n0 + wn * TN + j * 32 + 8 * g + 4 * fh;
          if (n >= p.N) continue;
          float v[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
          epilogue4<GLU, ACT>(p, C, R, m, n, v, b);
        }
    }
  }
}

// Fold split-K fp32 partials and apply the full epilogue; one thread per 4 columns.
template <bool GLU, int ACT>
__global__ void gemm_splitk_reduce(const GemmArgs p, const float* __restrict__ ws, int splits) {
  const int n4 = (p.N + 3) / 4;
  const long total = (long)p.M * n4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int m = (int)(i / n4);
    const int n = (int)(i - (long)m * n4) * 4;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (n + 3 < p.N && (p.N & 3) == 0) {
      // four partial slabs per round with every load issued before the first add (a dependent
      // load-add chain per split made the fold latency-bound: ~5 us for M = 64 decode GEMMs)
      const float* src = ws + (long)m * p.N + n;
      const long slab = (long)p.M * p.N;
      for (int s0 = 0; s0 < splits; s0 += 4) {
        float4_ x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          x[u] = s0 + u < splits ? *reinterpret_cast<const float4_*>(src + (s0 + u) * slab) : float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          v[0] += x[u][0]; v[1] += x[u][1]; v[2] += x[u][2]; v[3] += x[u][3];
        }
      }
    } else {
      for (int s = 0; s < splits; ++s) {
        const float* src = ws + (long)s * p.M * p.N + (long)m * p.N + n;
        for (int e = 0; e < 4 && n + e < p.N; ++e) v[e] += src[e];
      }
    }
    if (p.rms) {  // folded RMSNorm: per-row sum of squares partials follow the [splits][M][N] block
      const float* ss = ws + (long)splits * p.M * p.N;
      float t = 0.f;
      for (int s = 0; s < splits; ++s) t += ss[(long)s * p.M + m];
      const float r = rsqrtf(t / p.K + p.rms_eps);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] *= r;
    }
    // phase conv: row m's output pixel (no residual on that path)
    bf16_t* C = p.upsample == 2 ? p.C + (up2_out_row(p, m) - m) * p.ldc : p.C;
    epilogue4<GLU, ACT>(p, C, p.residual, m, n, v);
  }
}

// ---------------------------------------------------------------------------- dispatch
static int g_stages() {
  static int st = [] {
    const char* e = getenv("SHAI_GEMM_STAGES");
    return (e && e[0] == '3') ? 3 : 2;
  }();
  return st;
}

template <int BM, int BN, int WM, int WN, bool CONV, bool FAST, bool GLU, int ACT, bool SPLITK>
static void launch_cfg(const GemmArgs& a, float* ws, int splits, int kps, hipStream_t s, unsigned* cnt) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles, SPLITK ? splits : (a.batch > 0 ? a.batch : 1));
  if (g_stages() == 3 && (size_t)3 * (BM + BN) * BK2 * sizeof(bf16_t) <= 160 * 1024) {
    const size_t lds = (size_t)3 * (BM + BN) * BK2 * sizeof(bf16_t);
    gemm2_kernel<BM, BN, WM, WN, CONV, FAST, GLU, ACT, SPLITK, 3><<<grid, WM * WN * 64, lds, s>>>(a, ws, kps, cnt);
  } else {
    const size_t lds = (size_t)2 * (BM + BN) * BK2 * sizeof(bf16_t);
    gemm2_kernel<BM, BN, WM, WN, CONV, FAST, GLU, ACT, SPLITK, 2><<<grid, WM * WN * 64, lds, s>>>(a, ws, kps, cnt);
  }
}

// Tile configs: {BM, BN, WM, WN}.  256x320 covers the SD2.1 channel widths
// (320/640/1280/960/2560... are all multiples of 320) with no N waste and a
// 142 FLOP/B operand intensity; 256x256 for LLM / Flux widths.
struct TileCfg {
  int bm, bn;
  float eff;  // relative per-FLOP efficiency used by the planner
};
static const TileCfg kCfgs[] = {{256, 320, 1.00f}, {256, 256, 1.00f}, {256, 128, 0.90f}, {128, 128, 0.75f},
                                {128, 64, 0.55f}};
constexpr int kNumCfgs = 5;
// Config index space: [0, kNumCfgs) this file's tile configs; kNumCfgs + 0..3 the retired pipelined v3 kernel
// (cached choices run on v4); kNumCfgs + 4 / + 5 the 8-phase ping-pong v4 kernel (gemm_8ph.hip) with 256 / 320 wide tiles,
// kNumCfgs + 6 / + 7 the same in its persistent form (next tile's operands prefetched under the epilogue).
constexpr int kV4Cfg = kNumCfgs + 4;
// kV4Cfg + 4 / + 5: the four-wave kernel (gemm_w4.hip) with 256 x 256 / 192 x 320 tiles (128 x 128 / 96 x 160
// wave tiles; plain GEMM, GLU, conv; no split-K).
constexpr int kW4Cfg = kV4Cfg + 4;
// kW4Cfg + 2: the W-stationary low-K kernel (gemm_ws.hip): K = 320, N a multiple of 320, weights resident in VGPRs,
// persistent over M (plain / bias / act / GLU / residual / folded LayerNorm; no split-K).
constexpr int kWsCfg = kW4Cfg + 2;


template <bool CONV, bool FAST, bool GLU, int ACT>
static void launch_tiles(const GemmArgs& a, int cfg, float* ws, int splits, int kps, hipStream_t s, unsigned* cnt) {
  const bool sk = splits > 1;
#define SHAI_CFG(BM_, BN_, WM_, WN_)                                                   \
  if (sk) launch_cfg<BM_, BN_, WM_, WN_, CONV, FAST, GLU, ACT, true>(a, ws, splits, kps, s, cnt); \
  else launch_cfg<BM_, BN_, WM_, WN_, CONV, FAST, GLU, ACT, false>(a, ws, splits, kps, s, cnt);
  switch (cfg) {
    case 0: SHAI_CFG(256, 320, 4, 2); break;
    case 1: SHAI_CFG(256, 256, 4, 2); break;
    case 2: SHAI_CFG(256, 128, 4, 2); break;
    case 3: SHAI_CFG(128, 128, 2, 2); break;
    default: SHAI_CFG(128, 64, 2, 2); break;
  }
#undef SHAI_CFG
}

template <bool GLU, int ACT>
static void launch_reduce(const GemmArgs& a, const float* ws, int splits, hipStream_t s) {
  const long total = (long)a.M * ((a.N + 3) / 4);
  long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  gemm_splitk_reduce<GLU, ACT><<<(int)blocks, 256, 0, s>>>(a, ws, splits);
}

// Cost model: rounds of co-resident blocks x padded tile work / config efficiency.
// Blocks/CU from LDS (2 stages); 256 CUs.  Split-K only when the grid is small.
void gemm2_plan(const GemmArgs& a, int* cfg, int* splits) {
  const long M = a.M, N = a.N, K = a.K;
  const int batch = a.batch > 0 ? a.batch : 1;
  static const int forced = [] {
    const char* e = getenv("SHAI_GEMM_CFG");
    return e ? atoi(e) : -1;
  }();
  double best = 1e300;
  int bc = 3, bs = 1;
  const long kt = (K + BK2 - 1) / BK2;
  for (int c = 0; c < kNumCfgs; ++c) {
    if (forced >= 0 && c != forced) continue;
    const TileCfg& t = kCfgs[c];
    if (a.glu && (t.bn % 4)) continue;
    const long tm = (M + t.bm - 1) / t.bm, tn = (N + t.bn - 1) / t.bn;
    const long tiles = tm * tn * batch;
    const long lds = 2L * (t.bm + t.bn) * BK2 * 2;
    const long per_cu = std::max(1L, std::min(163840L / lds, 2048L / ((t.bm / 64) * (t.bn / 64) * 64 > 512 ? 512 : 256)));
    for (int sp = 1; sp <= 16; sp *= 2) {
      if (sp > 1 && (batch != 1 || kt / sp < 4)) break;
      const long blocks = tiles * sp;
      const long slots = 256 * per_cu;
      const long rounds = (blocks + slots - 1) / slots;
      const double work = (double)t.bm * t.bn * ((kt + sp - 1) / sp);
      double cost = rounds * work / t.eff;
      if (blocks < slots) cost *= 1.0 + 0.35 * (1.0 - (double)blocks / slots);  // idle CUs still cost latency
      if (sp > 1) cost += 0.02 * work * sp;                                   // partials + reduce pass
      if (cost < best) {
        best = cost;
        bc = c;
        bs = sp;
      }
    }
  }
  *cfg = bc;
  *splits = bs;
  // v4 (8-phase ping-pong) outruns every v2 tile on problems that fill the chip with 256-row tiles
  if (forced < 0 && gemm4_supported(a) && bs == 1) {
    const int bn = (N % 320 == 0 && N % 256 != 0) ? 320 : 256;
    const long tiles = ((M + 255) / 256) * ((N + bn - 1) / bn) * batch;
    if (tiles >= 192 && K >= 256) *cfg = kV4Cfg + (bn == 320 ? 1 : 0);
  }
}

size_t gemm2_workspace_bytes(const GemmArgs& a) {
  int cfg, splits;
  gemm2_plan(a, &cfg, &splits);
  return splits > 1 ? (size_t)splits * a.M * a.N * sizeof(float) : 0;
}

template <bool CONV, bool FAST>
static void launch_all(const GemmArgs& a, float* ws, int cfg, int splits, hipStream_t s) {
  if (ws == nullptr) splits = 1;
  const long kt = (a.K + BK2 - 1) / BK2;
  const int kps = (int)(((kt + splits - 1) / splits) * BK2);
  // split-K at the 256 x 128 / 128 x 64 tiles (cfg 2 / 4): fixed up inside the launch when a ticket slice is available
  // (SHAI_G2_FIXUP=0: the separate fold kernel)
  // Off by default: measured SLOWER end to end (SD2.1 bs1 p50 406 ms with it vs 356 ms with the fold kernel,
  // profiles/norm_handoff_round4.md): the write-through slabs and the last arriver's serial sum cost more than
  // the fold launch they replace.  SHAI_G2_FIXUP=1 enables it (tests force it through the forced-split hook).
  static const bool fixup_on = [] {
    const char* e = getenv("SHAI_G2_FIXUP");
    return e && e[0] == '1';
  }();
  unsigned* cnt = nullptr;
  // (not at 128 x 128: the fixup's registers would halve that config's occupancy)
  if (splits > 1 && (cfg == 2 || cfg == 4) && fixup_on && !a.rms && (long)splits * a.M * a.N * 4 < 0x7fffffffL) {
    const int bm = cfg == 2 ? 256 : 128, bn = cfg == 4 ? 64 : 128;
    const long tiles = (long)((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
    if (tiles <= 4096) cnt = skinny_ticket_slice(s, (int)tiles);
  }
#define SHAI_G2(GLU_, ACT_)                                                   \
  do {                                                                        \
    launch_tiles<CONV, FAST, GLU_, ACT_>(a, cfg, ws, splits, kps, s, cnt);    \
    if (splits > 1 && cnt == nullptr) launch_reduce<GLU_, ACT_>(a, ws, splits, s); \
  } while (0)
  if constexpr (CONV) {  // convs: no GLU, activation none / silu
    if (a.act == ACT_SILU) SHAI_G2(false, ACT_SILU);
    else SHAI_G2(false, ACT_NONE);
  } else if (a.glu) {
    if (a.act == ACT_SILU) SHAI_G2(true, ACT_SILU);
    else if (a.act == ACT_GELU_TANH) SHAI_G2(true, ACT_GELU_TANH);
    else SHAI_G2(true, ACT_GELU);
  } else {
    switch (a.act) {
      case ACT_SILU: SHAI_G2(false, ACT_SILU); break;
      case ACT_GELU: SHAI_G2(false, ACT_GELU); break;
      case ACT_GELU_TANH: SHAI_G2(false, ACT_GELU_TANH); break;
      case ACT_QUICK_GELU: SHAI_G2(false, ACT_QUICK_GELU); break;
      case ACT_RELU: SHAI_G2(false, ACT_RELU); break;
      default: SHAI_G2(false, ACT_NONE); break;
    }
  }
#undef SHAI_G2
}

void launch_gemm2_cfg(const GemmArgs& a, float* ws, int cfg, int splits, hipStream_t s) {
  if (cfg == kWsCfg) {  // whole K resident: a split-K choice is run unsplit
    launch_gemm_ws(a, s);
    return;
  }
  if (cfg == kW4Cfg || cfg == kW4Cfg + 1) {  // whole K per tile: a split-K choice is run unsplit
    launch_gemm_w4(a, cfg == kW4Cfg ? 256 : 320, s);
    return;
  }
  if (cfg >= kV4Cfg) {
    const int v = cfg - kV4Cfg;
    launch_gemm4(a, ws, splits, (v & 1) ? 320 : 256, s, v >= 2);
    return;
  }
  if (cfg >= kNumCfgs) {  // retired v3 (pipelined 256x256 / 256x320): a cached choice runs on v4, same tile width
    launch_gemm4(a, ws, splits, cfg - kNumCfgs >= 2 ? 320 : 256, s, false);
    return;
  }
  if (!a.conv) {
    launch_all<false, false>(a, ws, cfg, splits, s);
  } else {
    const bool fast = (a.Cin % 64) == 0 && (a.A2 == nullptr || (a.Cin1 % 64) == 0);
    if (fast) launch_all<true, true>(a, ws, cfg, splits, s);
    else launch_all<true, false>(a, ws, cfg, splits, s);
  }
}

// Split-K fold + full epilogue for fp32 partials laid out [splits][M][N] (also used by the skinny kernel).
void launch_splitk_epilogue(const GemmArgs& a, const float* ws, int splits, hipStream_t s) {
  if (a.glu) {  // every activation: the skinny kernels (any GLU activation) fold through here too
    switch (a.act) {
      case ACT_SILU: launch_reduce<true, ACT_SILU>(a, ws, splits, s); break;
      case ACT_GELU: launch_reduce<true, ACT_GELU>(a, ws, splits, s); break;
      case ACT_GELU_TANH: launch_reduce<true, ACT_GELU_TANH>(a, ws, splits, s); break;
      case ACT_QUICK_GELU: launch_reduce<true, ACT_QUICK_GELU>(a, ws, splits, s); break;
      case ACT_RELU: launch_reduce<true, ACT_RELU>(a, ws, splits, s); break;
      default: launch_reduce<true, ACT_NONE>(a, ws, splits, s); break;
    }
    return;
  }
  switch (a.act) {
    case ACT_SILU: launch_reduce<false, ACT_SILU>(a, ws, splits, s); break;
    case ACT_GELU: launch_reduce<false, ACT_GELU>(a, ws, splits, s); break;
    case ACT_GELU_TANH: launch_reduce<false, ACT_GELU_TANH>(a, ws, splits, s); break;
    case ACT_QUICK_GELU: launch_reduce<false, ACT_QUICK_GELU>(a, ws, splits, s); break;
    case ACT_RELU: launch_reduce<false, ACT_RELU>(a, ws, splits, s); break;
    default: launch_reduce<false, ACT_NONE>(a, ws, splits, s); break;
  }
}

int gemm2_num_cfgs() { return kWsCfg + 1; }

// Configs the autotuner races: not the retired v3 indices (kNumCfgs .. + 3; the pipelined kernel held 2 cached
// shapes when it was removed in round 5 -- every index stays valid for old caches) nor the lab-only 192 x 320
// four-wave tile.
bool gemm2_cfg_candidate(int cfg) { return !(cfg >= kNumCfgs && cfg < kV4Cfg) && cfg != kW4Cfg + 1; }

bool gemm2_cfg_splittable(int cfg) { return cfg != kW4Cfg && cfg != kW4Cfg + 1 && cfg != kWsCfg; }

bool gemm2_cfg_supported(const GemmArgs& a, int cfg) {
  // an epilogue activation no tile kernel instantiates is never accepted (it would run as another one)
  if (!tile_act_supported(a)) return false;
  // phase-decomposed upsample conv (upsample == 2) / weight slices: only the v4 kernel maps rows to output pixels
  // and tiles to weight slices
  if (a.upsample == 2 || a.w_slice_rows != 0) return cfg >= kV4Cfg && cfg < kV4Cfg + 4 && gemm4_supported(a);
  // folded LayerNorm (row_mr): only the v4 kernel's epilogue applies it, and only unsplit, batch 1
  if (a.row_mr != nullptr)
    return cfg == kWsCfg ? gemm_ws_supported(a) : cfg >= kV4Cfg && cfg < kV4Cfg + 4 && a.batch <= 1 && gemm4_supported(a);
  if (cfg == kWsCfg) return gemm_ws_supported(a);
  if (cfg == kW4Cfg) return gemm_w4_supported(a);
  if (cfg == kW4Cfg + 1) return false;  // 192 x 320 four-wave tile: lab only (gemm_w4.hip launch_gemm_w4)
  if (cfg >= kV4Cfg) return cfg < kV4Cfg + 4 && gemm4_supported(a);
  if (cfg >= kNumCfgs) return gemm4_supported(a);  // retired v3 -> v4
  if (a.in_scale != nullptr) return false;
  if (a.conv && a.A2 != nullptr && (a.Cin % 64 != 0 || a.Cin1 % 64 != 0)) return false;  // 64-wide K tiles
  return cfg >= 0 && cfg < kNumCfgs;
}

void gemm2_cfg_info(int cfg, int* bm, int* bn) {
  if (cfg == kWsCfg) {  // W-stationary kernel: reported as "1x-320"
    *bm = 1;
    *bn = -320;
    return;
  }
  if (cfg == kW4Cfg || cfg == kW4Cfg + 1) {  // four-wave kernel: reported as "4x-256" / "4x-320"
    *bm = 4;
    *bn = cfg == kW4Cfg ? -256 : -320;
    return;
  }
  if (cfg >= kV4Cfg) {  // 8-phase v4 kernel: reported as "8x-<BN>" ("9x-<BN>" persistent)
    *bm = cfg >= kV4Cfg + 2 ? 9 : 8;
    *bn = ((cfg - kV4Cfg) & 1) ? -320 : -256;
    return;
  }
  if (cfg >= kNumCfgs) {  // retired v3: runs as v4
    *bm = 8;
    *bn = cfg - kNumCfgs >= 2 ? -320 : -256;
    return;
  }
  *bm = kCfgs[cfg].bm;
  *bn = kCfgs[cfg].bn;
}

void launch_gemm2(const GemmArgs& a, float* ws, hipStream_t s) {
  int cfg, splits;
  gemm2_plan(a, &cfg, &splits);
  launch_gemm2_cfg(a, ws, cfg, splits, s);
}

}  // namespace shai
