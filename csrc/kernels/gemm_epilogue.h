// Shared GEMM epilogue (v2 LDS-DMA GEMM, pipelined 256x256 GEMM, split-K fold).
#pragma once
#include "common.h"
#include "launchers.h"

namespace shai {

// Phase-decomposed upsample conv (GemmArgs::upsample == 2, gemm_8ph.hip CONV 3), row order: groups of
// G = max(1, 256 / (H W)) images (H, W powers of two, host-checked); inside a group phase-major (ph = 2 py + px), then
// image, then (i, j) of the low-resolution grid.  A 256-row tile so holds ONE phase (its weight slice); G = 1 is
// image-major.  Shifts only: the epilogue evaluates this per stored row.
struct Up2Row {
  int img, ph, si, sj;
};
__device__ __forceinline__ Up2Row up2_row(const GemmArgs& p, int m) {
  const int lw = __builtin_ctz((unsigned)p.Wd), lhw = lw + __builtin_ctz((unsigned)p.H);
  const int lb = lhw >= 8 ? lhw : 8;  // log2 of one (group, phase) block's rows, G H W
  const int r = m & ((1 << lb) - 1), r2 = r & ((1 << lhw) - 1);
  Up2Row q;
  q.ph = (m >> lb) & 3;
  q.img = ((m >> (lb + 2)) << (lb - lhw)) + (r >> lhw);
  q.si = r2 >> lw;
  q.sj = r2 & (p.Wd - 1);
  return q;
}
// the output pixel row of GEMM row m (epilogue and split-K fold)
__device__ __forceinline__ long up2_out_row(const GemmArgs& p, int m) {
  const Up2Row q = up2_row(p, m);
  return ((long)q.img * p.OH + 2 * q.si + (q.ph >> 1)) * p.OW + 2 * q.sj + (q.ph & 1);
}

// Apply the epilogue to 4 consecutive columns n..n+3 of row m and store.
template <bool GLU, int ACT>
__device__ __forceinline__ void epilogue4(const GemmArgs& p, bf16_t* C, const bf16_t* R, int m, int n, float v[4],
                                          int b = 0) {
  const bool full = n + 3 < p.N && (p.ldc & 3) == 0 && (p.ldr & 3) == 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] *= p.alpha;
  if (p.bias) {
    if (full) {
      const uint2_ bb = *reinterpret_cast<const uint2_*>(p.bias + n);
      v[0] += bf2f(bb[0] & 0xffff); v[1] += bf2f(bb[0] >> 16);
      v[2] += bf2f(bb[1] & 0xffff); v[3] += bf2f(bb[1] >> 16);
    } else {
      for (int e = 0; e < 4 && n + e < p.N; ++e) v[e] += bf2f(p.bias[n + e]);
    }
  }
  if (p.bias2d) {
    const bf16_t* b2 = p.bias2d + (long)(m / p.rows_per_bias2d) * p.N;
    if (full && (p.N & 3) == 0) {
      const uint2_ bb = *reinterpret_cast<const uint2_*>(b2 + n);
      v[0] += bf2f(bb[0] & 0xffff); v[1] += bf2f(bb[0] >> 16);
      v[2] += bf2f(bb[1] & 0xffff); v[3] += bf2f(bb[1] >> 16);
    } else {
      for (int e = 0; e < 4 && n + e < p.N; ++e) v[e] += bf2f(b2[n + e]);
    }
  }
  const bf16_t* gr = p.gate ? p.gate + ((long)b * p.M + m) / p.rows_per_gate * p.gate_stride : nullptr;
  if constexpr (GLU) {
    float o0 = v[0] * apply_act<ACT>(v[1]);
    float o1 = v[2] * apply_act<ACT>(v[3]);
    const int nc = n >> 1;
    if (gr) {
      o0 *= bf2f(gr[nc]);
      o1 *= bf2f(gr[nc + 1]);
    }
    float r0 = 0.f, r1 = 0.f;
    if (R) {
      r0 = bf2f(R[(long)m * p.ldr + nc]) * p.res_alpha;
      r1 = bf2f(R[(long)m * p.ldr + nc + 1]) * p.res_alpha;
    }
    if (((p.ldc | nc) & 1) == 0) {
      *reinterpret_cast<uint32_t*>(C + (long)m * p.ldc + nc) = pack2(o0 + r0, o1 + r1);
    } else {
      C[(long)m * p.ldc + nc] = f2bf(o0 + r0);
      C[(long)m * p.ldc + nc + 1] = f2bf(o1 + r1);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = apply_act<ACT>(v[e]);
    if (gr) {
      for (int e = 0; e < 4 && n + e < p.N; ++e) v[e] *= bf2f(gr[n + e]);
    }
    if (full) {
      if (R) {
        const uint2_ rr = *reinterpret_cast<const uint2_*>(R + (long)m * p.ldr + n);
        v[0] += bf2f(rr[0] & 0xffff) * p.res_alpha; v[1] += bf2f(rr[0] >> 16) * p.res_alpha;
        v[2] += bf2f(rr[1] & 0xffff) * p.res_alpha; v[3] += bf2f(rr[1] >> 16) * p.res_alpha;
      }
      uint2_ o;
      o[0] = pack2(v[0], v[1]);
      o[1] = pack2(v[2], v[3]);
      *reinterpret_cast<uint2_*>(C + (long)m * p.ldc + n) = o;
    } else {
      for (int e = 0; e < 4 && n + e < p.N; ++e) {
        float x = v[e];
        if (R) x += bf2f(R[(long)m * p.ldr + n + e]) * p.res_alpha;
        C[(long)m * p.ldc + n + e] = f2bf(x);
      }
    }
  }
}

}  // namespace shai
