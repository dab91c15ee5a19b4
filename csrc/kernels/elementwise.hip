// Memory-bound elementwise kernels for gfx950 (16-byte bf16 vectors, grid
// capped at ~8 blocks/CU with grid-stride loops).
//   gated_act   : SwiGLU / GEGLU when the producing GEMM is not fused
//   bias_act    : bias + activation (+ residual)
//   rope        : rotary embedding (Llama/Mistral: neox halves; GPT-J: pairs)
//   rope_pairs  : Flux 3-axis RoPE from precomputed per-token cos/sin
//   sched_step  : classifier-free guidance + DDIM / Euler / flow-match update
//                 fused into one pass over the latents (the reference runs
//                 these as separate diffusers ops on host-driven tensors,
//                 app/run-sd.py:137-142, app/flux_model_api.py:146-211)
//   softmax     : row softmax (VAE mid-block attention fallback path)
//   embedding   : token embedding gather
#include "common.h"
#include "launchers.h"

namespace shai {

static inline int grid_for(long work, int block = 256) {
  long g = (work + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

__global__ void gated_act_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ out, long rows, int F, long xs,
                                 int act, int gate_first) {
  const int F8 = F >> 3;
  const long total = rows * F8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / F8;
    const int c = (int)(i - r * F8) * 8;
    const bf16_t* xr = x + r * xs;
    float a[8], g[8];
    unpack8(*reinterpret_cast<const uint4_*>(xr + c), a);
    unpack8(*reinterpret_cast<const uint4_*>(xr + F + c), g);
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = gate_first ? apply_act_rt(act, a[k]) * g[k] : a[k] * apply_act_rt(act, g[k]);
    *reinterpret_cast<uint4_*>(out + r * F + c) = pack8(o);
  }
}

void launch_gated_act(const bf16_t* x, bf16_t* out, long rows, int F, long x_stride, int act, int gate_first,
                      hipStream_t s) {
  gated_act_kernel<<<grid_for(rows * (F / 8)), 256, 0, s>>>(x, out, rows, F, x_stride, act, gate_first);
}

__global__ void bias_act_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ bias,
                                const bf16_t* __restrict__ res, bf16_t* __restrict__ out, long rows, int D, int act,
                                float alpha) {
  const int D8 = D >> 3;
  const long total = rows * D8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % D8) * 8;
    float f[8];
    unpack8(reinterpret_cast<const uint4_*>(x)[i], f);
    float bb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (bias) unpack8(*reinterpret_cast<const uint4_*>(bias + c), bb);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = apply_act_rt(act, f[k] * alpha + bb[k]);
    if (res) {
      float r[8];
      unpack8(reinterpret_cast<const uint4_*>(res)[i], r);
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] += r[k];
    }
    reinterpret_cast<uint4_*>(out)[i] = pack8(f);
  }
}

void launch_bias_act(const bf16_t* x, const bf16_t* bias, const bf16_t* residual, bf16_t* out, long rows, int D,
                     int act, float alpha, hipStream_t s) {
  bias_act_kernel<<<grid_for(rows * (D / 8)), 256, 0, s>>>(x, bias, residual, out, rows, D, act, alpha);
}

// x [T, H, Dh] (token stride ts), rotate the first rot_dim dims.
// neox: pairs (i, i + rot/2); else (2i, 2i+1).
__global__ void rope_kernel(bf16_t* __restrict__ x, const int* __restrict__ pos, const float* __restrict__ cs,
                            const float* __restrict__ sn, int T, int H, int Dh, int rot, long ts, int neox) {
  const int half = rot >> 1;
  const long total = (long)T * H * half;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int j = (int)(i % half);
    const int h = (int)((i / half) % H);
    const int t = (int)(i / ((long)half * H));
    bf16_t* xh = x + (long)t * ts + (long)h * Dh;
    const int p = pos[t];
    const float c = cs[(long)p * half + j], s = sn[(long)p * half + j];
    const int i0 = neox ? j : 2 * j, i1 = neox ? j + half : 2 * j + 1;
    const float a = bf2f(xh[i0]), b = bf2f(xh[i1]);
    xh[i0] = f2bf(a * c - b * s);
    xh[i1] = f2bf(b * c + a * s);
  }
}

void launch_rope(bf16_t* x, const int* positions, const float* cos, const float* sin, int T, int H, int Dh,
                 int rot_dim, long tok_stride, int neox, hipStream_t s) {
  rope_kernel<<<grid_for((long)T * H * (rot_dim / 2)), 256, 0, s>>>(x, positions, cos, sin, T, H, Dh, rot_dim,
                                                                     tok_stride, neox);
}

// Flux: x [B, T, H, Dh]; per (t, j) rotation of pair (2j, 2j+1) with cos/sin [T, Dh/2]
__global__ void rope_pairs_kernel(bf16_t* __restrict__ x, const float* __restrict__ cs, const float* __restrict__ sn,
                                  int B, int T, int H, int Dh, long bs, long ts) {
  const int half = Dh >> 1;
  const int q4 = half >> 2;  // 4 pairs (8 elements) per thread
  const long total = (long)B * T * H * q4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int j4 = (int)(i % q4);
    const int h = (int)((i / q4) % H);
    const int t = (int)((i / ((long)q4 * H)) % T);
    const int b = (int)(i / ((long)q4 * H * T));
    bf16_t* xp = x + (long)b * bs + (long)t * ts + (long)h * Dh + j4 * 8;
    float f[8];
    unpack8(*reinterpret_cast<const uint4_*>(xp), f);
    const float* c = cs + (long)t * half + j4 * 4;
    const float* s = sn + (long)t * half + j4 * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float a = f[2 * k], bb = f[2 * k + 1];
      f[2 * k] = a * c[k] - bb * s[k];
      f[2 * k + 1] = bb * c[k] + a * s[k];
    }
    *reinterpret_cast<uint4_*>(xp) = pack8(f);
  }
}

void launch_rope_pairs(bf16_t* x, const float* cos, const float* sin, int B, int T, int H, int Dh, long batch_stride,
                       long tok_stride, hipStream_t s) {
  rope_pairs_kernel<<<grid_for((long)B * T * H * (Dh / 8)), 256, 0, s>>>(x, cos, sin, B, T, H, Dh, batch_stride,
                                                                         tok_stride);
}

// latents [n] (bf16), model_out [2n] when cfg (uncond first) else [n]
// Per-row variant for step-level batching: latents [B, per_row] where every row (image) is at its own
// denoising step; rows[3 b .. 3 b + 2] = (a_t, a_prev, dt) of row b, a_t < 0 marks an idle row (left as is).
__global__ void sched_step_rows_kernel(const bf16_t* __restrict__ mo, bf16_t* __restrict__ lat, long n, long per_row,
                                       int cfg, float g, int pred, const float* __restrict__ rows) {
  const long n8 = n >> 3;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const long r = (i << 3) / per_row;
    const float a_t = rows[3 * r], a_prev = rows[3 * r + 1], dt = rows[3 * r + 2];
    if (a_t < 0.f) continue;
    float x[8], e[8];
    unpack8(reinterpret_cast<const uint4_*>(lat)[i], x);
    unpack8(reinterpret_cast<const uint4_*>(mo)[i], e);
    if (cfg) {
      float c[8];
      unpack8(reinterpret_cast<const uint4_*>(mo)[i + n8], c);
#pragma unroll
      for (int k = 0; k < 8; ++k) e[k] = e[k] + g * (c[k] - e[k]);
    }
    const float sa = sqrtf(a_t), s1a = sqrtf(1.f - a_t), sp = sqrtf(a_prev), s1p = sqrtf(1.f - a_prev);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (pred == 2) {
        x[k] = x[k] + dt * e[k];
      } else {
        float x0, eps;
        if (pred == 0) {
          eps = e[k];
          x0 = (x[k] - s1a * eps) / sa;
        } else {
          x0 = sa * x[k] - s1a * e[k];
          eps = sa * e[k] + s1a * x[k];
        }
        x[k] = sp * x0 + s1p * eps;
      }
    }
    reinterpret_cast<uint4_*>(lat)[i] = pack8(x);
  }
}

void launch_sched_step_rows(const bf16_t* mo, bf16_t* lat, long n, long per_row, int cfg, float g, int pred,
                            const float* rows, hipStream_t s) {
  sched_step_rows_kernel<<<grid_for(n / 8), 256, 0, s>>>(mo, lat, n, per_row, cfg, g, pred, rows);
}

__global__ void sched_step_kernel(const bf16_t* __restrict__ mo, bf16_t* __restrict__ lat, long n, int cfg,
                                  float g, int pred, float a_t, float a_prev, float dt) {
  const long n8 = n >> 3;
  const float sa = sqrtf(a_t), s1a = sqrtf(1.f - a_t);
  const float sp = sqrtf(a_prev), s1p = sqrtf(1.f - a_prev);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float x[8], e[8];
    unpack8(reinterpret_cast<const uint4_*>(lat)[i], x);
    unpack8(reinterpret_cast<const uint4_*>(mo)[i], e);
    if (cfg) {
      float c[8];
      unpack8(reinterpret_cast<const uint4_*>(mo)[i + n8], c);
#pragma unroll
      for (int k = 0; k < 8; ++k) e[k] = e[k] + g * (c[k] - e[k]);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (pred == 2) {  // flow matching Euler: x <- x + dt * v
        x[k] = x[k] + dt * e[k];
      } else {
        float x0, eps;
        if (pred == 0) {
          eps = e[k];
          x0 = (x[k] - s1a * eps) / sa;
        } else {  // v-prediction
          x0 = sa * x[k] - s1a * e[k];
          eps = sa * e[k] + s1a * x[k];
        }
        x[k] = sp * x0 + s1p * eps;
      }
    }
    reinterpret_cast<uint4_*>(lat)[i] = pack8(x);
  }
}

void launch_sched_step(const bf16_t* model_out, bf16_t* latents, long n, int cfg, float guidance, int pred_type,
                       float a_t, float a_prev, float dt, hipStream_t s) {
  sched_step_kernel<<<grid_for(n / 8), 256, 0, s>>>(model_out, latents, n, cfg, guidance, pred_type, a_t, a_prev, dt);
}

// one block (256 threads) per row
__global__ void softmax_kernel(bf16_t* __restrict__ x, int D, float scale) {
  __shared__ float red[8];
  bf16_t* row = x + (long)blockIdx.x * D;
  float m = -INFINITY;
  for (int c = threadIdx.x * 8; c < D; c += 256 * 8) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4_*>(row + c), f);
#pragma unroll
    for (int k = 0; k < 8; ++k) m = fmaxf(m, f[k] * scale);
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int c = threadIdx.x * 8; c < D; c += 256 * 8) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4_*>(row + c), f);
#pragma unroll
    for (int k = 0; k < 8; ++k) s += __expf(f[k] * scale - m);
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[4 + (threadIdx.x >> 6)] = s;
  __syncthreads();
  const float inv = 1.f / (red[4] + red[5] + red[6] + red[7]);
  for (int c = threadIdx.x * 8; c < D; c += 256 * 8) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4_*>(row + c), f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = __expf(f[k] * scale - m) * inv;
    *reinterpret_cast<uint4_*>(row + c) = pack8(f);
  }
}

void launch_softmax(bf16_t* x, long rows, int D, float scale, hipStream_t s) {
  softmax_kernel<<<(int)rows, 256, 0, s>>>(x, D, scale);
}

__global__ void embedding_kernel(const int* __restrict__ ids, const bf16_t* __restrict__ table,
                                 bf16_t* __restrict__ out, long T, int D) {
  const int D8 = D >> 3;
  const long total = T * D8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long t = i / D8;
    const int c = (int)(i - t * D8);
    reinterpret_cast<uint4_*>(out)[i] = reinterpret_cast<const uint4_*>(table + (long)ids[t] * D)[c];
  }
}

// Decode token feedback: ids[i] = prev[rowmap[i]] where rowmap[i] >= 0 (the previous decode step's sampled
// token of the same sequence, still on the device), else the host-supplied ids[i].
__global__ void token_feedback_kernel(int* __restrict__ ids, const int* __restrict__ rowmap,
                                      const int* __restrict__ prev, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int r = rowmap[i];
    if (r >= 0) ids[i] = prev[r];
  }
}

void launch_token_feedback(int* ids, const int* rowmap, const int* prev, int n, hipStream_t s) {
  token_feedback_kernel<<<(n + 255) / 256, 256, 0, s>>>(ids, rowmap, prev, n);
}

// Streams `bytes` of a scratch buffer through the cache hierarchy with plain loads (clean lines: no write-back
// traffic left behind), evicting whatever the Infinity Cache / L2 held.  The sum feeds a store that never
// happens (the data is zeros), so the loads are not dead.
__global__ void cache_flush_kernel(const uint4_* __restrict__ buf, long n, unsigned* __restrict__ sink) {
  unsigned acc = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const uint4_ v = buf[i];
    acc |= v.x | v.y | v.z | v.w;
  }
  if (acc == 0xdeadbeefu) sink[0] = acc;
}

void launch_cache_flush(const void* buf, size_t bytes, unsigned* sink, hipStream_t s) {
  cache_flush_kernel<<<2048, 256, 0, s>>>(reinterpret_cast<const uint4_*>(buf), (long)(bytes / 16), sink);
}

void launch_embedding(const int* ids, const bf16_t* table, bf16_t* out, long T, int D, hipStream_t s) {
  embedding_kernel<<<grid_for(T * (D / 8)), 256, 0, s>>>(ids, table, out, T, D);
}

}  // namespace shai
