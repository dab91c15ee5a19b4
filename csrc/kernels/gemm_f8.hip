// fp8 (OCP e4m3) MFMA GEMM for W8A8 prefill:
//
//   C[m, n] = epi(a_scale[m] * w_scale[n] * sum_k A8[m, k] * W8[n, k])     (epi: bias / act / GLU / residual)
//
// A8 is the activation quantised per row on the fly (quant_rows_fp8 below: absmax / 448, with the folded
// RMSNorm's rstd multiplied into the row scale), W8 the weight quantised per output row at load time
// (ops.quantize_fp8_rows).  The products run on v_mfma_scale_f32_32x32x64_f8f6f4 with unit block scales
// (E8M0 127): the 64-deep fp8 MFMA is the instruction that reaches gfx950's fp8 rate (the unscaled
// 32x32x16 fp8 form runs at the bf16 rate); the real scales are per row / per column and go to the epilogue.
//
// Structure (the bf16 LDS-DMA GEMM of gemm_lds.hip re-cut for 1-byte elements): a K step is 128 fp8 = one
// 128-byte row chunk per operand row, so the LDS image, the 8-row x 128-B DMA pieces and the XOR chunk
// swizzle are byte-for-byte those of the bf16 kernel at BK = 64.  Each lane's MFMA fragment is 32 bytes =
// two swizzled 16-B chunks of one row; A and W fragments use the same lane -> k map, so the k order inside
// a 64-deep step never matters.  Tiles BM x BN with WM x WN waves (each 64 x BN/WN of 32x32 blocks), three
// LDS stages, counted vmcnt + raw s_barrier (two tiles in flight while one is consumed), XCD-aware remap
// and grouped M order.
#include "common.h"
#include "launchers.h"
#include "gemm_epilogue.h"

namespace shai {

typedef int f8i32x8 __attribute__((ext_vector_type(8)));
typedef int f8i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void f8_lds_void;

constexpr int F8_BK = 128;           // fp8 elements (bytes) per K step and operand row
constexpr uint32_t F8_OOB = 0x80000000u;
constexpr int F8_E8M0_ONE = 127;     // block scale 2^0

__device__ __forceinline__ int f8_swz(int row, int ch) { return row * F8_BK + ((ch ^ ((row >> 1) & 7)) << 4); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t f8_rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)min(bytes, 0x7fffffffL),
                                           0x00020000);
}

__device__ __forceinline__ void f8_glds(__amdgpu_buffer_rsrc_t r, uint8_t* lds, uint32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (f8_lds_void*)lds, 16, off, 0, 0, 0);
}

template <int BM, int BN, int WM, int WN, bool GLU, int ACT, int STAGES>
__global__ void __launch_bounds__(WM * WN * 64) gemm_f8_kernel(const GemmArgs p, const uint8_t* __restrict__ A8,
                                                               const uint8_t* __restrict__ W8,
                                                               const float* __restrict__ a_scale,
                                                               const float* __restrict__ w_scale) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int IM = TM / 32, JN = TN / 32;
  constexpr int JA = BM / 8 / NW, JB = BN / 8 / NW;  // DMA wave-instructions per K step
  constexpr int PER = JA + JB;
  constexpr int STAGE = (BM + BN) * F8_BK;          // bytes per stage
  static_assert(JA >= 1 && JB >= 1 && IM >= 1 && JN >= 1, "bad tile config");
  extern __shared__ __attribute__((aligned(16))) uint8_t f8_smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;

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

  const __amdgpu_buffer_rsrc_t rA = f8_rsrc(A8, (long)p.M * p.lda);
  const __amdgpu_buffer_rsrc_t rW = f8_rsrc(W8, (long)p.N * p.ldw);
  const int lrow = lane >> 3, lpos = lane & 7;
  uint32_t a_off[JA], w_off[JB];
#pragma unroll
  for (int j = 0; j < JA; ++j) {
    const int r = (wid * JA + j) * 8 + lrow, m = m0 + r;
    a_off[j] = m < p.M ? (uint32_t)((long)m * p.lda + ((lpos ^ ((r >> 1) & 7)) << 4)) : F8_OOB;
  }
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    const int r = (wid * JB + j) * 8 + lrow, n = n0 + r;
    w_off[j] = n < p.N ? (uint32_t)((long)n * p.ldw + ((lpos ^ ((r >> 1) & 7)) << 4)) : F8_OOB;
  }
  auto stage = [&](int buf, int k0) {
    uint8_t* sa = f8_smem + buf * STAGE;
    uint8_t* sw = sa + BM * F8_BK;
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const int ch = lpos ^ ((((wid * JB + j) * 8 + lrow) >> 1) & 7);
      const uint32_t off = (w_off[j] != F8_OOB && k0 + ch * 16 < p.K) ? w_off[j] + (uint32_t)k0 : F8_OOB;
      f8_glds(rW, sw + (wid * JB + j) * 8 * F8_BK, off);
    }
#pragma unroll
    for (int j = 0; j < JA; ++j) {
      const int ch = lpos ^ ((((wid * JA + j) * 8 + lrow) >> 1) & 7);
      const uint32_t off = (a_off[j] != F8_OOB && k0 + ch * 16 < p.K) ? a_off[j] + (uint32_t)k0 : F8_OOB;
      f8_glds(rA, sa + (wid * JA + j) * 8 * F8_BK, off);
    }
  };

  float16_ acc[IM][JN];
#pragma unroll
  for (int i = 0; i < IM; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = (p.K + F8_BK - 1) / F8_BK;
  const int fr = lane & 31, fh = lane >> 5;
  auto frag = [&](const uint8_t* base, int row, int s) {  // 32 bytes: chunks 4s + 2fh, 4s + 2fh + 1
    const f8i32x4 lo = *reinterpret_cast<const f8i32x4*>(base + f8_swz(row, 4 * s + 2 * fh));
    const f8i32x4 hi = *reinterpret_cast<const f8i32x4*>(base + f8_swz(row, 4 * s + 2 * fh + 1));
    return f8i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  auto compute = [&](int buf) {
    const uint8_t* sa = f8_smem + buf * STAGE;
    const uint8_t* sw = sa + BM * F8_BK;
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // two 64-deep MFMA steps per 128-byte K step
      f8i32x8 af[IM], wf[JN];
#pragma unroll
      for (int i = 0; i < IM; ++i) af[i] = frag(sa, wm * TM + i * 32 + fr, s);
#pragma unroll
      for (int j = 0; j < JN; ++j) wf[j] = frag(sw, wn * TN + j * 32 + fr, s);
#pragma unroll
      for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wf[j], af[i], acc[i][j], 0, 0, 0, F8_E8M0_ONE,
                                                                      0, F8_E8M0_ONE);
    }
  };

  if constexpr (STAGES == 3) {
    // tiles t+1 and t+2 in flight while tile t is consumed (counted vmcnt retires this wave's DMA of tile t;
    // the raw barrier publishes every wave's part and frees tile t-1's buffer for tile t+2)
    if (nk > 0) stage(0, 0);
    if (nk > 1) stage(1, F8_BK);
    int buf = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + 2 < nk) stage(buf == 0 ? 2 : buf - 1, (kt + 2) * F8_BK);
      compute(buf);
      buf = buf == 2 ? 0 : buf + 1;
    }
  } else {
    // two stages (the 256 x 256 tile: 128 KB): tile t+1's DMA issued before tile t's MFMAs
    if (nk > 0) stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) stage((kt + 1) & 1, (kt + 1) * F8_BK);
      compute(kt & 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }

  // epilogue: lane owns row m (column of the swapped D), 4 groups of 4 consecutive n per 32x32 block
  const bf16_t* R = p.residual;
#pragma unroll
  for (int i = 0; i < IM; ++i) {
    const int m = m0 + wm * TM + i * 32 + fr;
    if (m >= p.M) continue;
    const float as = a_scale[m];
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wn * TN + j * 32 + 8 * g + 4 * fh;
        if (n >= p.N) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * g + e] * as * (n + e < p.N ? w_scale[n + e] : 0.f);
        epilogue4<GLU, ACT>(p, p.C, R, m, n, v, 0);
      }
  }
}

// ---- per-row activation quantisation: a8[m, :] = e4m3(x[m, :] / s[m]), s[m] = absmax / 448; with rms_eps >= 0
// the row's RMSNorm rstd (norm gain folded into the weights) is multiplied into the stored scale.  One workgroup
// per row: a statistics pass, then a conversion pass that re-reads the row (L2-resident).
__global__ void __launch_bounds__(256) quant_rows_fp8_kernel(const bf16_t* __restrict__ x, long ldx, int K,
                                                             uint8_t* __restrict__ out, long ldo,
                                                             float* __restrict__ scale, float rms_eps) {
  const int m = blockIdx.x, t = threadIdx.x;
  const bf16_t* xr = x + (long)m * ldx;
  float amax = 0.f, ss = 0.f;
  for (int k = t * 8; k < K; k += 256 * 8) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4_*>(xr + k), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      amax = fmaxf(amax, fabsf(v[e]));
      ss = fmaf(v[e], v[e], ss);
    }
  }
  __shared__ float red[2][4];
  amax = wave_max(amax);
  ss = wave_sum(ss);
  if ((t & 63) == 0) {
    red[0][t >> 6] = amax;
    red[1][t >> 6] = ss;
  }
  __syncthreads();
  amax = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
  ss = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  const float s = fmaxf(amax, 1e-30f) / 448.f;
  const float inv = 1.f / s;
  if (t == 0) scale[m] = rms_eps >= 0.f ? s * rsqrtf(ss / K + rms_eps) : s;
  uint8_t* orow = out + (long)m * ldo;
  for (int k = t * 8; k < K; k += 256 * 8) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4_*>(xr + k), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fminf(fmaxf(v[e] * inv, -448.f), 448.f);  // rounding never overflows e4m3
    int w0 = 0, w1 = 0;
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], w0, false);
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], w0, true);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], w1, false);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[6], v[7], w1, true);
    *reinterpret_cast<uint2_*>(orow + k) = uint2_{(uint32_t)w0, (uint32_t)w1};
  }
}

bool gemm_f8_supported(const GemmArgs& a) {
  return a.M >= 1 && a.N >= 1 && a.K % 16 == 0 && a.lda % 16 == 0 && a.ldw % 16 == 0 && !a.conv && a.batch <= 1 &&
         a.bias2d == nullptr && a.gate == nullptr && (!a.glu || a.N % 4 == 0) && (long)a.M * a.lda < 0x7fffffffL &&
         (long)a.N * a.ldw < 0x7fffffffL;
}

bool quant_rows_fp8_supported(int K) { return K % 8 == 0; }

void launch_quant_rows_fp8(const bf16_t* x, long ldx, int M, int K, uint8_t* out, long ldo, float* scale,
                           float rms_eps, hipStream_t s) {
  quant_rows_fp8_kernel<<<M, 256, 0, s>>>(x, ldx, K, out, ldo, scale, rms_eps);
}

// cfg 0: 256 x 128, 8 waves (4 x 2), 3 stages = 144 KB of LDS; cfg 1: 128 x 128, 4 waves (2 x 2), 96 KB;
// cfg 2: 256 x 256, 8 waves (2 x 4: 128 x 64 per wave, 0.75 fragment reads per MFMA), 2 stages = 128 KB
void launch_gemm_f8(const GemmArgs& a, const uint8_t* A8, const uint8_t* W8, const float* a_scale,
                    const float* w_scale, int cfg, hipStream_t s) {
#define F8L(BM, BN, WM, WN, G, A)                                                                               \
  gemm_f8_kernel<BM, BN, WM, WN, G, A, (BM + BN > 384 ? 2 : 3)>                                                 \
      <<<((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN), WM * WN * 64,                                          \
         (size_t)(BM + BN > 384 ? 2 : 3) * (BM + BN) * F8_BK, s>>>(a, A8, W8, a_scale, w_scale)
#define F8ACT(BM, BN, WM, WN, G)                          \
  switch (a.act) {                                        \
    case ACT_SILU: F8L(BM, BN, WM, WN, G, ACT_SILU); break; \
    case ACT_GELU: F8L(BM, BN, WM, WN, G, ACT_GELU); break; \
    case ACT_GELU_TANH: F8L(BM, BN, WM, WN, G, ACT_GELU_TANH); break; \
    case ACT_QUICK_GELU: F8L(BM, BN, WM, WN, G, ACT_QUICK_GELU); break; \
    case ACT_RELU: F8L(BM, BN, WM, WN, G, ACT_RELU); break; \
    default: F8L(BM, BN, WM, WN, G, ACT_NONE); break;     \
  }
  if (cfg == 0) {
    if (a.glu) { F8ACT(256, 128, 4, 2, true) } else { F8ACT(256, 128, 4, 2, false) }
  } else if (cfg == 2) {
    if (a.glu) { F8ACT(256, 256, 2, 4, true) } else { F8ACT(256, 256, 2, 4, false) }
  } else {
    if (a.glu) { F8ACT(128, 128, 2, 2, true) } else { F8ACT(128, 128, 2, 2, false) }
  }
#undef F8ACT
#undef F8L
}

}  // namespace shai
