// Normalisation kernels for gfx950: RMSNorm, LayerNorm (both with optional
// fused residual add) and channels-last GroupNorm (stats / finalize / apply).
//
// Row norms: one 64-lane wave owns one row, the row is held in registers as
// packed bf16 (16-byte vectors), so x is read once from HBM and written once.
// GroupNorm is split into a partial-statistics pass and a tiny finalize pass
// that emits per-(sample, channel) fp32 scale/shift.  The apply step is
// usually NOT a separate kernel: the implicit-GEMM conv kernel (conv.hip)
// applies scale/shift (+SiLU) while it gathers its A tile, so the normalised
// activation is never materialised (replaces the diffusers GroupNorm+SiLU
// pair the reference runs eagerly / via Inductor, app/run-sd.py:107-134).
#include "common.h"
#include "launchers.h"

namespace shai {

// ----------------------------------------------------------------------------
// RMSNorm / LayerNorm, one wave per row.
// ----------------------------------------------------------------------------
template <int MAXC, bool LAYERNORM>
__global__ void __launch_bounds__(256) row_norm_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ residual, const bf16_t* __restrict__ w,
    const bf16_t* __restrict__ b, bf16_t* __restrict__ out, bf16_t* __restrict__ residual_out, int rows,
    int D, long x_stride, long out_stride, float eps, float w_offset, int rows_per_w, long w_stride) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  if (rows_per_w > 0) {  // per-image modulation rows (AdaLN): w/b = row group of a strided [G, *] tensor
    const long wo = (long)(row / rows_per_w) * w_stride;
    if (w) w += wo;
    if (b) b += wo;
  }
  const bf16_t* xr = x + (long)row * x_stride;
  uint4_ v[MAXC];
  float sum = 0.f, sumsq = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < D) {
      v[c] = *reinterpret_cast<const uint4_*>(xr + col);
      if (residual) {
        const uint4_ r = *reinterpret_cast<const uint4_*>(residual + (long)row * D + col);
        float f[8], g[8];
        unpack8(v[c], f);
        unpack8(r, g);
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] += g[i];
        v[c] = pack8(f);
        if (residual_out) *reinterpret_cast<uint4_*>(residual_out + (long)row * D + col) = v[c];
      }
      float f[8];
      unpack8(v[c], f);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        sum += f[i];
        sumsq += f[i] * f[i];
      }
    }
  }
  float mean = 0.f, rstd;
  if (LAYERNORM) {
    mean = wave_sum(sum) / D;
    float var = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int col = (c * 64 + lane) * 8;
      if (col < D) {
        float f[8];
        unpack8(v[c], f);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float d = f[i] - mean;
          var += d * d;
        }
      }
    }
    rstd = rsqrtf(wave_sum(var) / D + eps);
  } else {
    rstd = rsqrtf(wave_sum(sumsq) / D + eps);
  }
  bf16_t* orow = out + (long)row * out_stride;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < D) {
      float f[8], wf[8], bf[8];
      unpack8(v[c], f);
      if (w) unpack8(*reinterpret_cast<const uint4_*>(w + col), wf);
      else
#pragma unroll
        for (int i = 0; i < 8; ++i) wf[i] = 1.f;
      if (LAYERNORM && b) unpack8(*reinterpret_cast<const uint4_*>(b + col), bf);
      else
#pragma unroll
        for (int i = 0; i < 8; ++i) bf[i] = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] = (f[i] - mean) * rstd * (wf[i] + w_offset) + bf[i];
      *reinterpret_cast<uint4_*>(orow + col) = pack8(f);
    }
  }
}

// Narrow rows (D <= 512, D % 64 == 0; e.g. the SD2.1 UNet's C = 320 LayerNorms over 262k rows):
// one wave row-per-wave left 24 of 64 lanes idle at D = 320 and paid a 6-step wave reduction per
// 640-B row.  Here 8 lanes own a row (8 rows per wave): each lane holds NV = D / 64 16-byte
// vectors (8-lane groups read 128 contiguous bytes per vector), reductions are 3 xor-shuffles.
template <int NV, bool LAYERNORM>
__global__ void __launch_bounds__(256) row_norm8_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ residual, const bf16_t* __restrict__ w,
    const bf16_t* __restrict__ b, bf16_t* __restrict__ out, bf16_t* __restrict__ residual_out, int rows,
    int D, long x_stride, long out_stride, float eps, float w_offset, int rows_per_w, long w_stride) {
  const int lane = threadIdx.x & 63, sub = lane & 7;
  const int row = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + (lane >> 3);
  const bool live = row < rows;
  const int r = live ? row : rows - 1;  // dead lanes mirror a real row (shuffles stay uniform)
  if (rows_per_w > 0) {
    const long wo = (long)(r / rows_per_w) * w_stride;
    if (w) w += wo;
    if (b) b += wo;
  }
  const bf16_t* xr = x + (long)r * x_stride;
  uint4_ v[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) v[c] = *reinterpret_cast<const uint4_*>(xr + (c * 8 + sub) * 8);
  if (residual) {
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int col = (c * 8 + sub) * 8;
      const uint4_ rr = *reinterpret_cast<const uint4_*>(residual + (long)r * D + col);
      float f[8], g[8];
      unpack8(v[c], f);
      unpack8(rr, g);
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] += g[i];
      v[c] = pack8(f);
      if (residual_out && live) *reinterpret_cast<uint4_*>(residual_out + (long)r * D + col) = v[c];
    }
  }
  float sum = 0.f, sumsq = 0.f;
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    float f[8];
    unpack8(v[c], f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sum += f[i];
      sumsq += f[i] * f[i];
    }
  }
#pragma unroll
  for (int m = 1; m < 8; m <<= 1) {
    sum += __shfl_xor(sum, m, 64);
    sumsq += __shfl_xor(sumsq, m, 64);
  }
  float mean = 0.f, rstd;
  if (LAYERNORM) {
    mean = sum / D;
    float var = 0.f;  // second pass over the registers (two-pass variance, as the wave-per-row kernel)
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      float f[8];
      unpack8(v[c], f);
#pragma unroll
      for (int i = 0; i < 8; ++i) var += (f[i] - mean) * (f[i] - mean);
    }
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) var += __shfl_xor(var, m, 64);
    rstd = rsqrtf(var / D + eps);
  } else {
    rstd = rsqrtf(sumsq / D + eps);
  }
  if (!live) return;
  bf16_t* orow = out + (long)r * out_stride;
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int col = (c * 8 + sub) * 8;
    float f[8], wf[8], bf[8];
    unpack8(v[c], f);
    if (w) unpack8(*reinterpret_cast<const uint4_*>(w + col), wf);
    else
#pragma unroll
      for (int i = 0; i < 8; ++i) wf[i] = 1.f;
    if (LAYERNORM && b) unpack8(*reinterpret_cast<const uint4_*>(b + col), bf);
    else
#pragma unroll
      for (int i = 0; i < 8; ++i) bf[i] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = (f[i] - mean) * rstd * (wf[i] + w_offset) + bf[i];
    *reinterpret_cast<uint4_*>(orow + col) = pack8(f);
  }
}

template <bool LN>
static void launch_row_norm(const RowNormArgs& a, hipStream_t s) {
  if (a.D % 64 == 0 && a.D <= 512 && a.x_stride % 8 == 0 && a.out_stride % 8 == 0 && a.rows > 0) {
    dim3 grid((a.rows + 31) / 32), block(256);  // 4 waves x 8 rows
#define SHAI_RN8(NV)                                                                                      \
  row_norm8_kernel<NV, LN><<<grid, block, 0, s>>>(a.x, a.residual, a.w, a.b, a.out, a.residual_out, a.rows, \
                                                  a.D, a.x_stride, a.out_stride, a.eps, a.w_offset,     \
                                                  a.rows_per_w, a.w_stride)
    switch (a.D / 64) {
      case 1: SHAI_RN8(1); break;
      case 2: SHAI_RN8(2); break;
      case 3: SHAI_RN8(3); break;
      case 4: SHAI_RN8(4); break;
      case 5: SHAI_RN8(5); break;
      case 6: SHAI_RN8(6); break;
      case 7: SHAI_RN8(7); break;
      default: SHAI_RN8(8); break;
    }
#undef SHAI_RN8
    return;
  }
  dim3 grid((a.rows + 3) / 4), block(256);
  const int chunks = (a.D + 511) / 512;
#define SHAI_RN(C)                                                                                       \
  row_norm_kernel<C, LN><<<grid, block, 0, s>>>(a.x, a.residual, a.w, a.b, a.out, a.residual_out, a.rows, \
                                                a.D, a.x_stride, a.out_stride, a.eps, a.w_offset, \
                                                a.rows_per_w, a.w_stride)
  if (chunks <= 1) SHAI_RN(1);
  else if (chunks <= 2) SHAI_RN(2);
  else if (chunks <= 4) SHAI_RN(4);
  else if (chunks <= 8) SHAI_RN(8);
  else SHAI_RN(16);
#undef SHAI_RN
}

void launch_rmsnorm(const RowNormArgs& a, hipStream_t s) { launch_row_norm<false>(a, s); }
void launch_layernorm(const RowNormArgs& a, hipStream_t s) { launch_row_norm<true>(a, s); }

// ----------------------------------------------------------------------------
// GroupNorm over channels-last [N, HW, C] (C % 8 == 0, C <= 4096).
// Pass 1: grid (N, NB); each block reduces a contiguous pixel range into
//         per-group (sum, sumsq) partials  -> part[N][NB][G][2].
// Pass 2: grid (N) -- or fused into pass 1's last block per image (ticket counters) --
//         reduce partials, emit scale/shift [N][C] (fp32) such that
//         y = x * scale + shift  ==  (x - mean) * rstd * gamma + beta.
// Pass 3 (optional): apply (+ SiLU) elementwise.
// ----------------------------------------------------------------------------
// Per-(image, group) finalize shared by the fused path (last stats block of an image) and the
// standalone kernel: reduce the NB partials of image n, emit scale/shift [C].
__device__ void gn_finalize_image(const float* __restrict__ part, const bf16_t* __restrict__ gamma,
                                  const bf16_t* __restrict__ beta, float* __restrict__ scale,
                                  float* __restrict__ shift, int n, int HW, int C, int G, int NB, float eps,
                                  bool coherent) {
  __shared__ float mean_s[128], rstd_s[128];
  __shared__ float red[2][256];
  const int Cg = C / G;
  // 256 threads = L lanes per group x G groups (L = 256 / G); lanes stride over the partials
  const int L = 256 / G;
  const int g0 = threadIdx.x % G, lane_k = threadIdx.x / G;
  float a = 0.f, b = 0.f;
  if (lane_k < L) {
    for (int k = lane_k; k < NB; k += L) {
      const float* src = part + (((long)n * NB + k) * G + g0) * 2;
      if (coherent) {  // written by other workgroups (possibly other XCDs) of this launch
        a += __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        b += __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        const float2 v = *reinterpret_cast<const float2*>(src);
        a += v.x;
        b += v.y;
      }
    }
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  __syncthreads();
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    double sa = 0.0, sb = 0.0;
    for (int l = 0; l < L; ++l) {
      sa += red[0][l * G + g];
      sb += red[1][l * G + g];
    }
    const double cnt = (double)HW * Cg;
    const double mean = sa / cnt;
    double var = sb / cnt - mean * mean;
    if (var < 0) var = 0;
    mean_s[g] = (float)mean;
    rstd_s[g] = (float)(1.0 / sqrt(var + (double)eps));
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int g = c / Cg;
    const float ga = gamma ? bf2f(gamma[c]) : 1.f;
    const float be = beta ? bf2f(beta[c]) : 0.f;
    const float sc = rstd_s[g] * ga;
    scale[(long)n * C + c] = sc;
    shift[(long)n * C + c] = be - mean_s[g] * sc;
  }
}

// Stats over channels-last [N, HW, C] whose channels [0, C1) come from x (row stride C1) and
// [C1, C) from x2 (row stride C - C1): the UNet up-block skip concat is never materialised.
// With `counters` the LAST block of image n (agent-scope ticket, self re-arming to 0 so a HIP
// graph replays it) also runs the finalize: one launch instead of stats + finalize.
__global__ void __launch_bounds__(256) gn_stats_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ x2,
                                                       int C1, float* __restrict__ part, int HW, int C, int G, int NB,
                                                       int ppb, unsigned* __restrict__ counters,
                                                       const bf16_t* __restrict__ gamma,
                                                       const bf16_t* __restrict__ beta, float* __restrict__ scale,
                                                       float* __restrict__ shift, float eps) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [P][C] sums then [P][C] sumsq
  const int n = blockIdx.y, blk = blockIdx.x;
  const int C8 = C >> 3;
  const int t = threadIdx.x;
  const int P = C8 <= 256 ? 256 / C8 : 1;
  const int p0 = blk * ppb;
  const int p1 = min(HW, p0 + ppb);
  const int C2 = C - C1;
  // each thread: pixel lane pl, channel vectors cv0 (and cv0+256 when C8>256)
  const int pl = C8 <= 256 ? t / C8 : 0;
  const int cv0 = C8 <= 256 ? t % C8 : t;
  const bool active = C8 <= 256 ? (t < P * C8) : (t < C8);
  const bool second = C8 > 256 && (t + 256) < C8;
  // per-thread source (x or x2) of its channel vector(s): base pointer + row stride
  auto src_of = [&](int cv, const bf16_t*& base, int& ld) {
    const int c = cv * 8;
    if (c < C1) {
      base = x + (long)n * HW * C1 + c;
      ld = C1;
    } else {
      base = x2 + (long)n * HW * C2 + (c - C1);
      ld = C2;
    }
  };
  const bf16_t* b0 = x;
  const bf16_t* b1 = x;
  int ld0 = C, ld1 = C;
  src_of(cv0, b0, ld0);
  if (second) src_of(cv0 + 256, b1, ld1);
  float s0[8], q0[8], s1[8], q1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s0[i] = q0[i] = s1[i] = q1[i] = 0.f;
  if (active) {
    int p = p0 + pl;
    // 4 independent 16-byte loads in flight per thread
    for (; p + 3 * P < p1; p += 4 * P) {
      uint4_ v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint4_*>(b0 + (long)(p + u * P) * ld0);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          s0[i] += f[i];
          q0[i] += f[i] * f[i];
        }
      }
      if (second) {
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint4_*>(b1 + (long)(p + u * P) * ld1);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float f[8];
          unpack8(v[u], f);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            s1[i] += f[i];
            q1[i] += f[i] * f[i];
          }
        }
      }
    }
    for (; p < p1; p += P) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4_*>(b0 + (long)p * ld0), f);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        s0[i] += f[i];
        q0[i] += f[i] * f[i];
      }
      if (second) {
        unpack8(*reinterpret_cast<const uint4_*>(b1 + (long)p * ld1), f);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          s1[i] += f[i];
          q1[i] += f[i] * f[i];
        }
      }
    }
  }
  float* ls = lds;
  float* lq = lds + P * C;
  if (active) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      ls[pl * C + cv0 * 8 + i] = s0[i];
      lq[pl * C + cv0 * 8 + i] = q0[i];
    }
    if (second) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        ls[(cv0 + 256) * 8 + i] = s1[i];
        lq[(cv0 + 256) * 8 + i] = q1[i];
      }
    }
  }
  __syncthreads();
  // reduce over pixel lanes into row 0
  for (int c = t; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int p = 0; p < P; ++p) {
      a += ls[p * C + c];
      b += lq[p * C + c];
    }
    ls[c] = a;
    lq[c] = b;
  }
  __syncthreads();
  const int Cg = C / G;
  for (int g = t; g < G; g += 256) {
    float a = 0.f, b = 0.f;
    for (int c = 0; c < Cg; ++c) {
      a += ls[g * Cg + c];
      b += lq[g * Cg + c];
    }
    float* o = part + (((long)n * NB + blk) * G + g) * 2;
    if (counters) {  // read back by another workgroup of this launch: store at agent scope
      __hip_atomic_store(o, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(o + 1, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      o[0] = a;
      o[1] = b;
    }
  }
  if (!counters) return;
  // Fence-free hand-off (MI355X_MICROARCH.md, sc1 hand-off table, row 1): partials stored sc1
  // (agent-scope relaxed stores above), every storing wave waits for its stores, a barrier, then
  // ONE lane's agent-scope add; the block whose add returns NB-1 reads every partial with sc1
  // loads.  No buffer_wbl2 / buffer_inv (an acq_rel fence per block measured 2x slower).
  __shared__ unsigned s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const unsigned prev = __hip_atomic_fetch_add(counters + n, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == (unsigned)(NB - 1);
    if (s_last) __hip_atomic_store(counters + n, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  }
  __syncthreads();
  if (!s_last) return;
  gn_finalize_image(part, gamma, beta, scale, shift, n, HW, C, G, NB, eps, true);
}

__global__ void __launch_bounds__(256) gn_finalize_kernel(const float* __restrict__ part, const bf16_t* __restrict__ gamma,
                                                          const bf16_t* __restrict__ beta, float* __restrict__ scale,
                                                          float* __restrict__ shift, int HW, int C, int G, int NB,
                                                          float eps) {
  gn_finalize_image(part, gamma, beta, scale, shift, blockIdx.x, HW, C, G, NB, eps, false);
}

// Apply pass, y = (silu)(x * scale[n, c] + shift[n, c]) over channels-last [N, HW, C] (two sources: channels
// [0, C1) from x, [C1, C) from x2).  The launcher makes the grid's thread count a multiple of C / 8, so every
// thread keeps ONE 8-channel vector for the whole grid-stride loop: its scale / shift (4 x 16 B) are loaded once
// per image instead of once per 16 B of x, and the pixel index advances by a constant -- no 64-bit division per
// element group (both dominated the old loop's issue).
__global__ void __launch_bounds__(256) gn_apply_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ x2,
                                                       int C1, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, bf16_t* __restrict__ out,
                                                       long total8, int HW, int C, int silu) {
  const int C8 = C >> 3, C18 = C1 >> 3, C28 = (C - C1) >> 3;
  const long stride = (long)gridDim.x * blockDim.x;  // a multiple of C8
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= total8) return;
  const int cv = (int)(i % C8);
  long pix = i / C8;
  const long pstep = stride / C8;
  int n = (int)(pix / HW);
  long next = (long)(n + 1) * HW;
  const bool first = cv < C18;
  const uint4_* src = first ? reinterpret_cast<const uint4_*>(x) + cv : reinterpret_cast<const uint4_*>(x2) + (cv - C18);
  const int srcw = first ? C18 : C28;
  float4_ a0, a1, b0, b1;
  auto load_ss = [&]() {
    const float* sc = scale + (long)n * C + cv * 8;
    const float* sh = shift + (long)n * C + cv * 8;
    a0 = *reinterpret_cast<const float4_*>(sc);
    a1 = *reinterpret_cast<const float4_*>(sc + 4);
    b0 = *reinterpret_cast<const float4_*>(sh);
    b1 = *reinterpret_cast<const float4_*>(sh + 4);
  };
  load_ss();
  for (; i < total8; i += stride, pix += pstep) {
    if (pix >= next) {  // crossed into another image (rare unless HW is small)
      n = (int)(pix / HW);
      next = (long)(n + 1) * HW;
      load_ss();
    }
    float f[8];
    unpack8(src[pix * srcw], f);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[k] = f[k] * a0[k] + b0[k];
      f[k + 4] = f[k + 4] * a1[k] + b1[k];
    }
    if (silu)
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = silu_f(f[k]);
    reinterpret_cast<uint4_*>(out)[i] = pack8(f);
  }
}

int gn_num_blocks(int N, int HW, int C) {
  // Enough blocks to cover the chip (>= ~2048 workgroups over 256 CUs; 256 pixels/block left the
  // 16x16x1280 UNet levels on 16 CUs), but each block still reduces >= 16 KB so the per-block LDS
  // reduction stays amortised.  At most 256 partial slots per sample (finalize / workspace bound).
  const long bytes = (long)HW * C * 2;
  int by_size = (int)(bytes / (16 << 10));
  int want = (2048 + N - 1) / N;
  int nb = want < by_size ? want : by_size;
  if (nb > HW) nb = HW;
  if (nb > 256) nb = 256;
  if (nb < 1) nb = 1;
  return nb;
}

void launch_groupnorm_stats(const GroupNormArgs& a, hipStream_t s) {
  const int NB = gn_num_blocks(a.N, a.HW, a.C);
  const int ppb = (a.HW + NB - 1) / NB;
  const int C8 = a.C / 8;
  const int P = C8 <= 256 ? 256 / C8 : 1;
  const size_t lds = (size_t)2 * P * a.C * sizeof(float);
  const int C1 = a.x2 ? a.C1 : a.C;
  gn_stats_kernel<<<dim3(NB, a.N), 256, lds, s>>>(a.x, a.x2, C1, a.partials, a.HW, a.C, a.G, NB, ppb, a.counters,
                                                  a.gamma, a.beta, a.scale, a.shift, a.eps);
  if (!a.counters)
    gn_finalize_kernel<<<a.N, 256, 0, s>>>(a.partials, a.gamma, a.beta, a.scale, a.shift, a.HW, a.C, a.G, NB, a.eps);
}

void launch_groupnorm_apply(const GroupNormArgs& a, hipStream_t s) {
  const long total8 = (long)a.N * a.HW * a.C / 8;
  long blocks = (total8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  // grid threads a multiple of C / 8 (the kernel keeps one channel vector per thread)
  const int C8 = a.C / 8;
  int g = C8, b = 256;
  while (b) { const int t = g % b; g = b; b = t; }  // gcd(C8, 256)
  const long unit = C8 / g;
  blocks = (blocks + unit - 1) / unit * unit;
  gn_apply_kernel<<<(int)blocks, 256, 0, s>>>(a.x, a.x2, a.x2 ? a.C1 : a.C, a.scale, a.shift, a.out, total8, a.HW,
                                              a.C, a.silu);
}


// ---------------------------------------------------------------------------------------------------------------
// Norm statistics handed from a GEMM epilogue to the next norm (GemmArgs::col_part / row_part, gemm_8ph.hip), and
// the passes that produce the same statistics when the producing kernel could not (fallbacks).

// col partials [M / 128, N, 2] of x [M, N]: block = 128 rows x 64 channel vectors (512 channels); 256 threads =
// 64 vectors x 4 row lanes, each lane 32 rows with 8 independent 16-B loads in flight (batch-1 steps give only a
// few 128-row blocks, so the per-thread loop must not be latency-bound)
__global__ void __launch_bounds__(256) col_partials_kernel(const bf16_t* __restrict__ x, long M, int N, long ldx,
                                                           float* __restrict__ part) {
  __shared__ float4_ red[4][64][4];  // [row lane][vector][sum 0-3, sum 4-7, sq 0-3, sq 4-7]
  const int C8 = N >> 3, t = threadIdx.x;
  const int v = t & 63, rl = t >> 6;
  const int cv = blockIdx.y * 64 + v;
  const long r0 = (long)blockIdx.x * 128 + rl * 32;
  float s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = q[e] = 0.f;
  if (cv < C8) {
    const bf16_t* src = x + r0 * ldx + cv * 8;
#pragma unroll
    for (int r8 = 0; r8 < 32; r8 += 8) {
      uint4_ u[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        u[k] = r0 + r8 + k < M ? *reinterpret_cast<const uint4_*>(src + (long)(r8 + k) * ldx) : uint4_{0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float f[8];
        unpack8(u[k], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s[e] += f[e];
          q[e] = fmaf(f[e], f[e], q[e]);
        }
      }
    }
  }
  red[rl][v][0] = float4_{s[0], s[1], s[2], s[3]};
  red[rl][v][1] = float4_{s[4], s[5], s[6], s[7]};
  red[rl][v][2] = float4_{q[0], q[1], q[2], q[3]};
  red[rl][v][3] = float4_{q[4], q[5], q[6], q[7]};
  __syncthreads();
  if (rl == 0 && cv < C8) {
    float4_ a0 = red[0][v][0], a1 = red[0][v][1], b0 = red[0][v][2], b1 = red[0][v][3];
#pragma unroll
    for (int l = 1; l < 4; ++l) {
      a0 += red[l][v][0];
      a1 += red[l][v][1];
      b0 += red[l][v][2];
      b1 += red[l][v][3];
    }
    float4_* dst = reinterpret_cast<float4_*>(part + ((long)blockIdx.x * N + cv * 8) * 2);
    dst[0] = float4_{a0[0], b0[0], a0[1], b0[1]};
    dst[1] = float4_{a0[2], b0[2], a0[3], b0[3]};
    dst[2] = float4_{a1[0], b1[0], a1[1], b1[1]};
    dst[3] = float4_{a1[2], b1[2], a1[3], b1[3]};
  }
}

void launch_col_partials(const bf16_t* x, long M, int N, long ldx, float* part, hipStream_t s) {
  if (M <= 0) return;
  const int C8 = N >> 3;
  col_partials_kernel<<<dim3((unsigned)((M + 127) / 128), (C8 + 63) / 64), 256, 0, s>>>(x, M, N, ldx, part);
}

// GroupNorm (scale, shift) from the col partials of x (channels [0, C1)) and x2 ([C1, C1 + C2)): one wave per
// (image, group) sums the group's HW / 128 x C / G partial pairs (double), then writes its channels' scale / shift
__global__ void __launch_bounds__(64) gn_from_partials_kernel(const float* __restrict__ part1, int C1,
                                                              const float* __restrict__ part2, int C2, int HW, int G,
                                                              const bf16_t* __restrict__ gamma,
                                                              const bf16_t* __restrict__ beta, float eps,
                                                              float* __restrict__ scale, float* __restrict__ shift) {
  const int n = blockIdx.x, g = blockIdx.y, lane = threadIdx.x;
  const int C = C1 + C2, R = HW / 128, Cg = C / G, c0 = g * Cg;
  double a = 0.0, b = 0.0;
  for (int e = lane; e < R * Cg; e += 64) {
    const int r = e / Cg, c = c0 + (e - r * Cg);
    const float2 v = c < C1 ? *reinterpret_cast<const float2*>(part1 + (((long)n * R + r) * C1 + c) * 2)
                            : *reinterpret_cast<const float2*>(part2 + (((long)n * R + r) * C2 + (c - C1)) * 2);
    a += v.x;
    b += v.y;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  const double cnt = (double)HW * Cg;
  const double mean = a / cnt;
  double var = b / cnt - mean * mean;
  if (var < 0) var = 0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps)), m = (float)mean;
  for (int c = c0 + lane; c < c0 + Cg; c += 64) {
    const float sc = rstd * (gamma ? bf2f(gamma[c]) : 1.f);
    scale[(long)n * C + c] = sc;
    shift[(long)n * C + c] = (beta ? bf2f(beta[c]) : 0.f) - m * sc;
  }
}

void launch_gn_from_partials(const float* part1, int C1, const float* part2, int C2, int Nimg, int HW, int G,
                             const bf16_t* gamma, const bf16_t* beta, float eps, float* scale, float* shift,
                             hipStream_t s) {
  gn_from_partials_kernel<<<dim3(Nimg, G), 64, 0, s>>>(part1, C1, part2, C2, HW, G, gamma, beta, eps, scale, shift);
}

// LayerNorm row moments (mean, rstd) from the per-row partials of a GEMM epilogue: one thread per row
__global__ void __launch_bounds__(256) row_moments_part_kernel(const float* __restrict__ part, long M, int slots,
                                                               float inv_n, float eps, float* __restrict__ mr) {
  const long m = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (m >= M) return;
  // slot k holds (mean_k, M2_k) of its N / slots columns (equal counts): Chan's combination, no E[x^2] - mean^2
  const float2* src = reinterpret_cast<const float2*>(part) + m * slots;
  float a = 0.f;
  for (int k = 0; k < slots; ++k) a += src[k].x;
  const float mean = a / slots;
  float m2 = 0.f;
  for (int k = 0; k < slots; ++k) {
    const float2 v = src[k];
    const float d = v.x - mean;
    m2 += v.y + d * d * (1.f / (inv_n * slots));  // n_k = N / slots
  }
  const float var = fmaxf(m2 * inv_n, 0.f);
  *reinterpret_cast<float2*>(mr + 2 * m) = make_float2(mean, rsqrtf(var + eps));
}

void launch_row_moments_from_partials(const float* part, long M, int slots, int N, float eps, float* mr,
                                      hipStream_t s) {
  if (M <= 0) return;
  row_moments_part_kernel<<<(unsigned)((M + 255) / 256), 256, 0, s>>>(part, M, slots, 1.f / N, eps, mr);
}

// the same moments straight from x [M, N] (fallback): one wave per row, lanes over 8-element vectors
__global__ void __launch_bounds__(256) row_moments_kernel(const bf16_t* __restrict__ x, long M, int N, long ldx,
                                                          float eps, float* __restrict__ mr) {
  const long m = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (m >= M) return;
  // sums shifted by the row's first value: no catastrophic cancellation for rows with |mean| >> std
  const float k0 = bf2f(x[m * ldx]);
  float a = 0.f, b = 0.f;
  for (int c = lane * 8; c < N; c += 512) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4_*>(x + m * ldx + c), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = f[e] - k0;
      a += d;
      b = fmaf(d, d, b);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  if (lane == 0) {
    const float ms = a / N;
    const float var = fmaxf(b / N - ms * ms, 0.f);
    *reinterpret_cast<float2*>(mr + 2 * m) = make_float2(k0 + ms, rsqrtf(var + eps));
  }
}

void launch_row_moments(const bf16_t* x, long M, int N, long ldx, float eps, float* mr, hipStream_t s) {
  if (M <= 0) return;
  row_moments_kernel<<<(unsigned)((M + 3) / 4), 256, 0, s>>>(x, M, N, ldx, eps, mr);
}

}  // namespace shai
