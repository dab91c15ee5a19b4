// bf16 GEMM / implicit-GEMM convolution, v3: deep LDS-DMA pipeline, 256x256 tile.
//
//   C[b,m,n] = gate * act(alpha * sum_k A[b,m,k] * W[b,n,k] + bias[n] + bias2d) + res_alpha * Res[b,m,n]
//
// Why a third kernel: the v2 kernel (gemm_lds.hip) is the classic 2-buffer loop --
// one `vmcnt(0)` + barrier per K-tile -- and that structure tops out around
// 0.85 PF on this chip because every K-step waits for its own tile's DMA.  Here the
// staging ring is 4 deep and the DMA of three future K-tiles stays in flight ACROSS
// the barriers:
//
// * 256x256 output tile, 8 waves (2 along M x 4 along N), each wave 128x64 =
//   8x4 blocks of v_mfma_f32_16x16x32_bf16 (W fragment as the A operand so each
//   lane ends up owning 4 consecutive output columns of one row -> 8-byte stores).
// * BK = 32: a K-step's A and W tiles are 256 rows x 64 B each (32 KB per stage),
//   filled by 4 `buffer_load ... lds` (16 B / lane) per thread; 4 stages = 128 KB.
// * Per K-step: counted `s_waitcnt vmcnt(4 x tiles-still-allowed-in-flight)` (never
//   0 in steady state), raw `s_barrier` (NOT __syncthreads, whose fence would drain
//   the DMA queue), refill the ring slot of step t-1 with step t+3, then 12
//   ds_read_b128 fragments and 32 MFMAs under s_setprio(1).
// * LDS image lane-linear per wave instruction (16 rows x 64 B); the bank swizzle
//   (16-B chunk ^= (row >> 2) & 3) is applied to the per-lane SOURCE address and
//   to the ds_read address -> conflict-free 16-lane groups (16 distinct rows).
// * Range-checked buffer descriptors give the zero fill for M/N/K tails and conv
//   padding; XCD-aware bijective block remap + grouped M ordering as in v2.
// * Implicit-GEMM conv when Cin (and the concat split Cin1) are multiples of 32:
//   each 32-wide K-step then lies inside one filter tap, so the tap is uniform per
//   step and only the (ih, iw) of the lane's two rows are computed per step.
#include "gemm_epilogue.h"

namespace shai {

typedef __bf16 bf16x8p __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void g3_lds_void;

constexpr int G3_BM = 256, G3_BK = 32;
// BN = 256: 8 waves of 128x64; BN = 320 (every SD2.1 UNet channel count is a multiple of 320, so no
// N-tile waste): 8 waves of 128x80, the extra 64 W rows staged by waves 0-3 (5 DMAs per step for
// those waves, 4 for the others -- the counted vmcnt waits are per-wave constants).
template <int BN>
struct G3 {
  static constexpr int STAGE = (G3_BM + BN) * G3_BK;  // elements per ring slot (32 / 36 KB)
  static constexpr int NJ = BN / 64;                  // 16-column MFMA blocks per wave (4 / 5)
  static constexpr int WN_COLS = BN / 4;              // columns per wave (64 / 80)
};
constexpr uint32_t G3_OOB = 0x80000000u;

__device__ __forceinline__ int g3_swz(int row, int ch) { return row * G3_BK + ((ch ^ ((row >> 2) & 3)) << 3); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t g3_rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)min(bytes, 0x7fffffffL),
                                           0x00020000);
}

__device__ __forceinline__ void g3_glds(__amdgpu_buffer_rsrc_t r, bf16_t* lds, uint32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (g3_lds_void*)lds, 16, off, 0, 0, 0);
}

template <bool CONV, bool GLU, int ACT, bool SPLITK, int G3_STAGES, int G3_BN>
__global__ void __launch_bounds__(512) gemm3_kernel(const GemmArgs p, float* __restrict__ ws, int k_per_split) {
  constexpr int G3_STAGE = G3<G3_BN>::STAGE, NJ = G3<G3_BN>::NJ, WC = G3<G3_BN>::WN_COLS;
  extern __shared__ __attribute__((aligned(16))) bf16_t g3_smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;

  // ---- tile mapping (XCD remap + grouped M ordering)
  const int tiles_m = (p.M + G3_BM - 1) / G3_BM, tiles_n = (p.N + G3_BN - 1) / G3_BN;
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
  const int m0 = (first_m + in_group % gsize) * G3_BM;
  const int n0 = (in_group / gsize) * G3_BN;
  const int b = SPLITK ? 0 : blockIdx.y;
  const int kz = SPLITK ? blockIdx.y : 0;
  const int k_begin = kz * k_per_split;
  const int k_end = min(p.K, k_begin + k_per_split);

  const bf16_t* A = p.A + (long)b * p.batch_a;
  const bf16_t* Wt = p.W + (long)b * p.batch_w;
  const __amdgpu_buffer_rsrc_t rW = g3_rsrc(Wt, (long)p.N * p.ldw * 2);
  __amdgpu_buffer_rsrc_t rA, rA2;
  if constexpr (CONV) {
    rA = g3_rsrc(A, (long)p.Nimg * p.H * p.Wd * (p.A2 ? p.Cin1 : p.Cin) * 2);
    rA2 = p.A2 ? g3_rsrc(p.A2, (long)p.Nimg * p.H * p.Wd * (p.Cin - p.Cin1) * 2) : rA;
  } else {
    rA = g3_rsrc(A, (long)p.M * p.lda * 2);
    rA2 = rA;
  }

  // ---- staging geometry: wave instruction j fills 16 LDS rows x 64 B (lane-linear)
  const int lrow = lane >> 2, lpos = lane & 3;
  int row_j[2], ch_j[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    row_j[j] = (wid * 2 + j) * 16 + lrow;
    ch_j[j] = lpos ^ ((row_j[j] >> 2) & 3);
  }
  const int xrow = 256 + wid * 16 + lrow;             // BN = 320: this wave's extra W row
  const int xch = lpos ^ ((xrow >> 2) & 3);
  int cn[2] = {0, 0}, coh[2] = {0, 0}, cow[2] = {0, 0};
  bool cvalid[2] = {false, false};
  if constexpr (CONV) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = m0 + row_j[j];
      cvalid[j] = m < p.M;
      const int mm = cvalid[j] ? m : 0;
      const int hw = p.OH * p.OW;
      cn[j] = mm / hw;
      const int rem = mm - cn[j] * hw;
      coh[j] = rem / p.OW;
      cow[j] = rem - coh[j] * p.OW;
    }
  }

  auto stage = [&](int buf, int k0) {
    bf16_t* sa = g3_smem + buf * G3_STAGE;
    bf16_t* sw = sa + G3_BM * G3_BK;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + row_j[j], k = k0 + ch_j[j] * 8;
      const uint32_t off = (n < p.N && k < k_end) ? (uint32_t)(((long)n * p.ldw + k) * 2) : G3_OOB;
      g3_glds(rW, sw + (wid * 2 + j) * 16 * G3_BK, off);
    }
    if constexpr (G3_BN == 320) {
      if (wid < 4) {  // W rows 256 + 16 wid .. +15
        const int n = n0 + xrow, k = k0 + xch * 8;
        const uint32_t off = (n < p.N && k < k_end) ? (uint32_t)(((long)n * p.ldw + k) * 2) : G3_OOB;
        g3_glds(rW, sw + (256 + wid * 16) * G3_BK, off);
      }
    }
    if constexpr (!CONV) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int m = m0 + row_j[j], k = k0 + ch_j[j] * 8;
        const uint32_t off = (m < p.M && k < k_end) ? (uint32_t)(((long)m * p.lda + k) * 2) : G3_OOB;
        g3_glds(rA, sa + (wid * 2 + j) * 16 * G3_BK, off);
      }
    } else {
      // K-step lies inside one tap (Cin % 32 == 0): tap, channel base and source tensor are uniform
      const int tap = k0 / p.Cin;
      const int c0 = k0 - tap * p.Cin;
      const bool second = p.A2 != nullptr && c0 >= p.Cin1;
      const int kh = tap / p.KW, kw = tap - kh * p.KW;
      const int cs = p.A2 ? (second ? p.Cin - p.Cin1 : p.Cin1) : p.Cin;
      const int cb = second ? c0 - p.Cin1 : c0;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        int ih, iw;
        bool ok = cvalid[j] && k0 < k_end;
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
        const uint32_t off =
            ok ? (uint32_t)(((((long)cn[j] * p.H + ih) * p.Wd + iw) * cs + cb + ch_j[j] * 8) * 2) : G3_OOB;
        g3_glds(second ? rA2 : rA, sa + (wid * 2 + j) * 16 * G3_BK, off);
      }
    }
  };

  float4_ acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = float4_{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto compute = [&](int buf) {
    const bf16_t* sa = g3_smem + buf * G3_STAGE;
    const bf16_t* sw = sa + G3_BM * G3_BK;
    bf16x8p af[8], wf[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) wf[j] = *reinterpret_cast<const bf16x8p*>(sw + g3_swz(wn * WC + j * 16 + fr, fq));
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = *reinterpret_cast<const bf16x8p*>(sa + g3_swz(wm * 128 + i * 16 + fr, fq));
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = k_end > k_begin ? (k_end - k_begin + G3_BK - 1) / G3_BK : 0;
#pragma unroll
  for (int i = 0; i < G3_STAGES - 1; ++i)
    if (i < nk) stage(i, k_begin + i * G3_BK);
  for (int kt = 0; kt < nk; ++kt) {
    // retire this thread's DMA of step kt; steps kt+1, kt+2 may stay in flight
    const int ahead = min(G3_STAGES - 2, nk - 1 - kt);
    if (G3_BN == 320 && wid < 4) {  // 5 DMAs per step for these waves
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // everyone's step-kt DMA landed; everyone is done reading step kt-1
    if (kt + G3_STAGES - 1 < nk) stage((kt + G3_STAGES - 1) % G3_STAGES, k_begin + (kt + G3_STAGES - 1) * G3_BK);
    compute(kt % G3_STAGES);
  }

  // ---- epilogue: D[n][m] blocks -> lane owns row m = fr, columns n..n+3 = 4 fq + reg
  if constexpr (SPLITK) {
    float* Wp = ws + (long)kz * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wm * 128 + i * 16 + fr;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = n0 + wn * WC + j * 16 + 4 * fq;
        if (n + 3 < p.N) {
          *reinterpret_cast<float4_*>(Wp + (long)m * p.N + n) = acc[i][j];
        } else {
          for (int e = 0; e < 4 && n + e < p.N; ++e) Wp[(long)m * p.N + n + e] = acc[i][j][e];
        }
      }
    }
  } else {
    bf16_t* __restrict__ C = p.C + (long)b * p.batch_c;
    const bf16_t* __restrict__ R = p.residual ? p.residual + (long)b * p.batch_r : nullptr;
    const bool fast = m0 + G3_BM <= p.M && n0 + G3_BN <= p.N && p.bias2d == nullptr && p.gate == nullptr &&
                      (p.ldc & 3) == 0 && (R == nullptr || (p.ldr & 3) == 0);
    if (fast) {
      // Interior tile: per-column bias hoisted (4 column groups per lane), every residual load
      // issued before any store, so the tail waits once instead of once per 4 outputs.
      const bf16_t* __restrict__ bias = p.bias;
      float bj[NJ][4];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = n0 + wn * WC + j * 16 + 4 * fq;
        if (bias) {
          const uint2_ bb = *reinterpret_cast<const uint2_*>(bias + n);
          bj[j][0] = bf2f(bb[0] & 0xffff); bj[j][1] = bf2f(bb[0] >> 16);
          bj[j][2] = bf2f(bb[1] & 0xffff); bj[j][3] = bf2f(bb[1] >> 16);
        } else {
          bj[j][0] = bj[j][1] = bj[j][2] = bj[j][3] = 0.f;
        }
      }
      // residual rows are prefetched in groups of IG row blocks: all 8 at NJ = 4 (the tail waits
      // once); 2 at NJ = 5, where the 160 accumulator registers leave no room for 80 more
      constexpr int IG = NJ == 4 ? 8 : 2;
      if constexpr (!GLU) {
#pragma unroll
        for (int i0 = 0; i0 < 8; i0 += IG) {
        uint2_ rr[IG][NJ];
        if (R) {
#pragma unroll
          for (int ii = 0; ii < IG; ++ii)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              rr[ii][j] = *reinterpret_cast<const uint2_*>(R + (long)(m0 + wm * 128 + (i0 + ii) * 16 + fr) * p.ldr +
                                                           n0 + wn * WC + j * 16 + 4 * fq);
        }
#pragma unroll
        for (int ii = 0; ii < IG; ++ii) {
          const int i = i0 + ii;
          const int m = m0 + wm * 128 + i * 16 + fr;
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int n = n0 + wn * WC + j * 16 + 4 * fq;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = apply_act<ACT>(acc[i][j][e] * p.alpha + bj[j][e]);
            if (R) {
              v[0] += bf2f(rr[ii][j][0] & 0xffff) * p.res_alpha; v[1] += bf2f(rr[ii][j][0] >> 16) * p.res_alpha;
              v[2] += bf2f(rr[ii][j][1] & 0xffff) * p.res_alpha; v[3] += bf2f(rr[ii][j][1] >> 16) * p.res_alpha;
            }
            uint2_ o;
            o[0] = pack2(v[0], v[1]);
            o[1] = pack2(v[2], v[3]);
            *reinterpret_cast<uint2_*>(C + (long)m * p.ldc + n) = o;
          }
        }
        }
      } else {
#pragma unroll
        for (int i0 = 0; i0 < 8; i0 += IG) {
        uint32_t rr[IG][NJ];
        if (R) {
#pragma unroll
          for (int ii = 0; ii < IG; ++ii)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              rr[ii][j] = *reinterpret_cast<const uint32_t*>(R + (long)(m0 + wm * 128 + (i0 + ii) * 16 + fr) * p.ldr +
                                                            ((n0 + wn * WC + j * 16 + 4 * fq) >> 1));
        }
#pragma unroll
        for (int ii = 0; ii < IG; ++ii) {
          const int i = i0 + ii;
          const int m = m0 + wm * 128 + i * 16 + fr;
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int nc = (n0 + wn * WC + j * 16 + 4 * fq) >> 1;
            float o0 = (acc[i][j][0] * p.alpha + bj[j][0]) * apply_act<ACT>(acc[i][j][1] * p.alpha + bj[j][1]);
            float o1 = (acc[i][j][2] * p.alpha + bj[j][2]) * apply_act<ACT>(acc[i][j][3] * p.alpha + bj[j][3]);
            if (R) {
              o0 += bf2f(rr[ii][j] & 0xffff) * p.res_alpha;
              o1 += bf2f(rr[ii][j] >> 16) * p.res_alpha;
            }
            *reinterpret_cast<uint32_t*>(C + (long)m * p.ldc + nc) = pack2(o0, o1);
          }
        }
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wm * 128 + i * 16 + fr;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = n0 + wn * WC + j * 16 + 4 * fq;
        if (n >= p.N) continue;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        epilogue4<GLU, ACT>(p, C, R, m, n, v, b);
      }
    }
  }
}

// ---------------------------------------------------------------------------- host side
bool gemm3_supported(const GemmArgs& a) {
  if (a.in_scale != nullptr) return false;
  if (a.conv) {
    if (a.Cin % 32 != 0) return false;
    if (a.A2 != nullptr && a.Cin1 % 32 != 0) return false;
  }
  return true;
}

template <bool CONV, bool GLU, int ACT, int BN>
static void g3_launch_bn(const GemmArgs& a, float* ws, int splits, int kps, int stages, hipStream_t s) {
  const int tiles = ((a.M + G3_BM - 1) / G3_BM) * ((a.N + BN - 1) / BN);
  // 4-stage ring (128 / 144 KB, 1 workgroup / CU, 3 K-steps in flight) for long K; 2-stage ring
  // (64 / 72 KB, 2 workgroups / CU, so one tile's prologue / epilogue overlaps the other's main loop).
  const size_t lds = (size_t)stages * G3<BN>::STAGE * sizeof(bf16_t);
  dim3 grid(tiles, splits > 1 ? splits : (a.batch > 0 ? a.batch : 1));
  if (stages == 4) {
    if (splits > 1) gemm3_kernel<CONV, GLU, ACT, true, 4, BN><<<grid, 512, lds, s>>>(a, ws, kps);
    else gemm3_kernel<CONV, GLU, ACT, false, 4, BN><<<grid, 512, lds, s>>>(a, ws, kps);
  } else {
    if (splits > 1) gemm3_kernel<CONV, GLU, ACT, true, 2, BN><<<grid, 512, lds, s>>>(a, ws, kps);
    else gemm3_kernel<CONV, GLU, ACT, false, 2, BN><<<grid, 512, lds, s>>>(a, ws, kps);
  }
}

template <bool CONV, bool GLU, int ACT>
static void g3_launch(const GemmArgs& a, float* ws, int splits, int kps, int stages, int bn, hipStream_t s) {
  if (bn == 320) g3_launch_bn<CONV, GLU, ACT, 320>(a, ws, splits, kps, stages, s);
  else g3_launch_bn<CONV, GLU, ACT, 256>(a, ws, splits, kps, stages, s);
}

// splits > 1 requires ws ([splits][M][N] fp32); the caller runs launch_splitk_epilogue afterwards.
void launch_gemm3(const GemmArgs& a, float* ws, int splits, int stages, hipStream_t s, int bn) {
  if (ws == nullptr) splits = 1;
  const long kt = (a.K + G3_BK - 1) / G3_BK;
  const int kps = (int)(((kt + splits - 1) / splits) * G3_BK);
  if (a.conv) {
    if (a.act == ACT_SILU) g3_launch<true, false, ACT_SILU>(a, ws, splits, kps, stages, bn, s);
    else g3_launch<true, false, ACT_NONE>(a, ws, splits, kps, stages, bn, s);
  } else if (a.glu) {
    if (a.act == ACT_SILU) g3_launch<false, true, ACT_SILU>(a, ws, splits, kps, stages, bn, s);
    else if (a.act == ACT_GELU_TANH) g3_launch<false, true, ACT_GELU_TANH>(a, ws, splits, kps, stages, bn, s);
    else g3_launch<false, true, ACT_GELU>(a, ws, splits, kps, stages, bn, s);
  } else {
    switch (a.act) {
      case ACT_SILU: g3_launch<false, false, ACT_SILU>(a, ws, splits, kps, stages, bn, s); break;
      case ACT_GELU: g3_launch<false, false, ACT_GELU>(a, ws, splits, kps, stages, bn, s); break;
      case ACT_GELU_TANH: g3_launch<false, false, ACT_GELU_TANH>(a, ws, splits, kps, stages, bn, s); break;
      case ACT_QUICK_GELU: g3_launch<false, false, ACT_QUICK_GELU>(a, ws, splits, kps, stages, bn, s); break;
      case ACT_RELU: g3_launch<false, false, ACT_RELU>(a, ws, splits, kps, stages, bn, s); break;
      default: g3_launch<false, false, ACT_NONE>(a, ws, splits, kps, stages, bn, s); break;
    }
  }
  if (splits > 1) launch_splitk_epilogue(a, ws, splits, s);
}

}  // namespace shai
