// Diffusion-transformer (Flux MMDiT) helpers.
//
//   qk_norm_rope : per-head RMSNorm of Q and K (norm_q / norm_k, and the
//                  norm_added_* pair for the text stream) fused with the
//                  3-axis pair RoPE, in place on the packed QKV projection
//                  output [rows, 3, H, D].  One wave per (row, head, q|k);
//                  with D = 128 each lane owns exactly one rotation pair, so
//                  the sum of squares is one wave reduction and the rotation
//                  needs no cross-lane traffic.  Replaces three separate
//                  passes (norm_q, norm_k, apply_rotary_emb) in diffusers'
//                  FluxAttnProcessor (reference: app/src/transformer/model.py
//                  runs them inside the traced NEFF).
#include "common.h"
#include "launchers.h"

namespace shai {

__global__ void __launch_bounds__(256) qk_norm_rope_kernel(bf16_t* __restrict__ x, long ld, int rows, int S, int H,
                                                           int D, const bf16_t* __restrict__ qw,
                                                           const bf16_t* __restrict__ kw, const float* __restrict__ cs,
                                                           const float* __restrict__ sn, float eps) {
  const int lane = threadIdx.x & 63;
  const long item = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= (long)rows * H * 2) return;
  const int which = (int)(item & 1);
  const int h = (int)((item >> 1) % H);
  const long r = item / (2L * H);
  const int half = D >> 1;
  bf16_t* p = x + r * ld + (long)which * H * D + (long)h * D;
  const bool act = lane < half;
  float f0 = 0.f, f1 = 0.f;
  if (act) {
    const uint32_t u = *reinterpret_cast<const uint32_t*>(p + 2 * lane);
    f0 = bf2f(u & 0xffff);
    f1 = bf2f(u >> 16);
  }
  const bf16_t* w = which ? kw : qw;
  if (w) {
    const float rstd = rsqrtf(wave_sum(f0 * f0 + f1 * f1) / D + eps);
    if (act) {
      const uint32_t wu = *reinterpret_cast<const uint32_t*>(w + 2 * lane);
      f0 *= rstd * bf2f(wu & 0xffff);
      f1 *= rstd * bf2f(wu >> 16);
    }
  }
  if (!act) return;
  if (cs) {
    const long t = r % S;
    const float c = cs[t * half + lane], s = sn[t * half + lane];
    const float a = f0, b = f1;
    f0 = a * c - b * s;
    f1 = b * c + a * s;
  }
  *reinterpret_cast<uint32_t*>(p + 2 * lane) = pack2(f0, f1);
}

void launch_qk_norm_rope(bf16_t* x, long ld, int rows, int S, int H, int D, const bf16_t* qw, const bf16_t* kw,
                         const float* cs, const float* sn, float eps, hipStream_t s) {
  const long items = (long)rows * H * 2;
  qk_norm_rope_kernel<<<(unsigned)((items + 3) / 4), 256, 0, s>>>(x, ld, rows, S, H, D, qw, kw, cs, sn, eps);
}

}  // namespace shai
