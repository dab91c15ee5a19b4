// Shared GEMM epilogue (v2 LDS-DMA GEMM, pipelined 256x256 GEMM, split-K fold).
#pragma once
#include "common.h"
#include "launchers.h"

namespace shai {

// Phase-decomposed upsample conv (GemmArgs::upsample == 2, gemm_8ph.hip CONV 3): the output pixel row of GEMM row m
// (rows ordered image, phase, i, j over the low-resolution grid) -- the split-K fold's row map.
__device__ __forceinline__ long up2_out_row(const GemmArgs& p, int m) {
  const int hwl = p.H * p.Wd, ohw = p.OH * p.OW;
  const int cn = m / ohw, rem = m - cn * ohw;
  const int ph = rem / hwl, r2 = rem - ph * hwl;
  const int si = r2 / p.Wd, sj = r2 - si * p.Wd;
  return (long)cn * ohw + (long)(2 * si + (ph >> 1)) * p.OW + 2 * sj + (ph & 1);
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
