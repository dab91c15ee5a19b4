// Skinny GEMM for decode-shaped problems (M <= 64 activation rows: LLM decode
// batches, per-request modulation GEMMs):
//
//   C[m, n] = act(alpha * sum_k X[m, k] * W[n, k] + bias[n]) (+ res_alpha * R[m, n]),  GLU optional
//
// Purely weight-bandwidth bound, so the design goal is "keep enough bytes of W
// in flight per CU to cover HBM latency" (Little's law: ~8 TB/s x ~2 us over 256
// CUs is ~64 KB per CU), with every global load fully coalesced:
//
// * Workgroup = 4 waves, tile = 64 W rows (n) x all M rows of X (one 32-row
//   group for M <= 32, two for M <= 64), walking its K range in 64-wide steps.
//   Each step's W tile (8 KB) and X tile (4 / 8 KB) move global -> LDS with
//   buffer_load ... lds DMA (8 full 128 B rows per wave instruction; range
//   check = zero fill for X rows >= M / W rows >= N), through a ring of
//   6 x 12 KB (MB = 32) or 4 x 16 KB (MB = 64, two workgroups per CU), so
//   several steps are always in flight while one is consumed.  Counted vmcnt +
//   one s_barrier per step (same protocol as the GEMM in gemm_lds.hip).
// * Wave w consumes the 16-wide K slice [16w, 16w + 16) of each step: 32x32x16
//   MFMAs with W rows 0-31 / 32-63 as A and each 32-row X group (transposed) as
//   B, so one W fragment feeds both X groups -- at M = 64 the weights are still
//   streamed exactly once.  XOR-swizzled LDS image (source-side swizzle,
//   conflict-free ds_read_b128).
// * Cross-wave reduction through LDS, fused epilogue (bias / act / GLU /
//   residual / folded RMSNorm).  When N/64 tiles cannot fill the chip, K is
//   additionally split over KG workgroups writing fp32 partials that the shared
//   split-K fold (gemm_lds.hip) reduces + epilogues.
// * fp8 weights (F8, GemmArgs::w_scale set): W is OCP e4m3 [N, K] with one fp32 scale per
//   output row.  The W tile is 64 rows x 64 B (one DMA instruction per wave, 16-B chunk
//   swizzle chunk ^ (row >> 2) & 3); each lane's 8-byte fragment is widened in registers
//   (v_cvt_pk_f32_fp8 -> bf16, exact) and fed to the same bf16 MFMA; the row scale is applied
//   in the reduction.  Half the weight bytes per token: decode is weight-bandwidth bound.
#include "common.h"
#include "launchers.h"
#include "gemm_epilogue.h"

#include <cstdlib>
#include <map>
#include <mutex>

namespace shai {

typedef __bf16 bf16x8s __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void sk_lds_void;

constexpr int SK_BN = 64;       // W rows per workgroup
constexpr int SK_BK = 64;       // K per step
constexpr int SK_WAVES = 4;
constexpr uint32_t SK_OOB = 0x80000000u;
constexpr int SK_RP4 = SK_BN + 4;  // floats per m row of the cross-wave reduction image (16 B of bank skew)

// (An X-in-registers variant with an 8-deep W-only ring measured 10-25 % slower at M = 64 --
// profiles/mistral7b_b64_async_decode_round2.md -- and was dropped: the X tile in LDS is not the limiter.)
template <int MB, bool F8 = false>
struct SkGeom {
  static constexpr int XG = MB / 32;                    // 32-row X groups
  static constexpr int STAGES = MB == 32 ? 6 : 4;
  static constexpr int W_ELEMS = F8 ? SK_BN * SK_BK / 2 : SK_BN * SK_BK;  // W tile in bf16 units
  static constexpr int STAGE_ELEMS = W_ELEMS + MB * SK_BK;  // W tile then X tile
  static constexpr int PER = (F8 ? 1 : 2) + XG;         // DMA instructions per wave per step
  static constexpr size_t RED = (size_t)SK_WAVES * MB * SK_RP4 * 4;  // reduction image red[w][m][n]
  static constexpr size_t LDS = (size_t)STAGES * STAGE_ELEMS * 2 > RED ? (size_t)STAGES * STAGE_ELEMS * 2 : RED;
};

__device__ __forceinline__ int sk_swz(int row, int ch) { return row * SK_BK + ((ch ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t sk_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// write-through (sc1) 4-byte store / load for the in-kernel split-K hand-off (cache policy bit sc1 = 16)
__device__ __forceinline__ void sk_store_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)off, 0, 16);
}
__device__ __forceinline__ float sk_load_wt(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 16));
}

// the same, 16 B per lane (the slab of the in-launch split-K fixup, one float4 per thread and quad)
__device__ __forceinline__ void sk_store_wt4(__amdgpu_buffer_rsrc_t r, uint32_t off, const float v[4]) {
  const uint4_ u = uint4_{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
  __builtin_amdgcn_raw_buffer_store_b128(u, r, (int)off, 0, 16);
}
__device__ __forceinline__ float4_ sk_load_wt4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float4_, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16));
}

template <int PER, int N>
__device__ __forceinline__ void sk_wait_upto(int pending) {
  // s_waitcnt needs an immediate: allow `pending` DMA groups (of PER loads) to stay in flight
  if constexpr (N == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (pending >= N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N * PER) : "memory");
    else sk_wait_upto<PER, N - 1>(pending);
  }
}

template <bool GLU, int ACT>
__device__ __forceinline__ void sk_store(const GemmArgs& p, int n, int m, float v0, float v1) {
  if (n >= p.N) return;
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

// 8 fp8 (e4m3) weights at `src` (8-byte aligned LDS) -> bf16x8 (exact widening)
__device__ __forceinline__ bf16x8s sk_fp8x8(const bf16_t* src) {
  const uint2_ v = *reinterpret_cast<const uint2_*>(src);
  bf16x8s r;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)v[h], false);
    const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)v[h], true);
    r[4 * h + 0] = (__bf16)lo[0];
    r[4 * h + 1] = (__bf16)lo[1];
    r[4 * h + 2] = (__bf16)hi[0];
    r[4 * h + 3] = (__bf16)hi[1];
  }
  return r;
}

// byte offset of the 8-byte chunk c8 (0..7) of fp8 W row `row` in the 64 x 64 B tile image
__device__ __forceinline__ int sk_f8_off(int row, int c8) {
  return row * 64 + (((c8 >> 1) ^ ((row >> 2) & 3)) << 4) + ((c8 & 1) << 3);
}

template <int MB, bool GLU, int ACT, bool RMS, bool F8>
__global__ void __launch_bounds__(SK_WAVES * 64) skinny_gemm_kernel(const GemmArgs p, float* __restrict__ ws,
                                                                    int kg_steps, unsigned* __restrict__ cnt) {
  using G = SkGeom<MB, F8>;
  constexpr int XG = G::XG;
  extern __shared__ __attribute__((aligned(16))) bf16_t sk_smem[];
  __shared__ float ss_red[SK_WAVES][64 * XG];
  __shared__ float rstd_s[MB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tile = blockIdx.x, kg = blockIdx.y, KG = gridDim.y;
  const int n0 = tile * SK_BN;

  const int ksteps = (p.K + SK_BK - 1) / SK_BK;
  const int t0 = kg * kg_steps;
  const int nk = max(0, min(ksteps, t0 + kg_steps) - t0);

  const __amdgpu_buffer_rsrc_t rW = sk_rsrc(p.W, (uint32_t)min((long)p.N * p.ldw * (F8 ? 1 : 2), 0x7fffffffL));
  const __amdgpu_buffer_rsrc_t rX = sk_rsrc(p.A, (uint32_t)min((long)p.M * p.lda * 2, 0x7fffffffL));

  // DMA geometry: a wave instruction fills 8 LDS rows x 128 B, lane-linear; the lane at
  // LDS chunk position lpos fetches global chunk lpos ^ swz(row).
  const int lrow = lane >> 3, lpos = lane & 7;
  int wr[2], wc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    wr[j] = (w * 2 + j) * 8 + lrow;
    wc[j] = lpos ^ ((wr[j] >> 1) & 7);
  }
  const int xr = w * 8 + lrow;                 // X rows xr (+ 32 for the second group)
  const int xc = lpos ^ ((xr >> 1) & 7);       // (xr + 32) has the same swizzle

  // fp8 W: one wave instruction = 16 rows x 64 B; lane at chunk position lpos4 fetches chunk lpos4 ^ swz
  const int f8row = w * 16 + (lane >> 2), f8pos = lane & 3;
  const int f8c = f8pos ^ ((f8row >> 2) & 3);
  auto stage = [&](int buf, int step) {
    bf16_t* sw = sk_smem + buf * G::STAGE_ELEMS;
    bf16_t* sx = sw + G::W_ELEMS;
    const int k0 = (t0 + step) * SK_BK;
    if constexpr (F8) {
      const int n = n0 + f8row, k = k0 + f8c * 16;
      const uint32_t off = (n < p.N && k < p.K) ? (uint32_t)((long)n * p.ldw + k) : SK_OOB;
      if (p.w_nt) __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (sk_lds_void*)(sw + w * 16 * 32), 16, off, 0, 0, 2);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (sk_lds_void*)(sw + w * 16 * 32), 16, off, 0, 0, 0);
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wr[j], k = k0 + wc[j] * 8;
        const uint32_t off = (n < p.N && k < p.K) ? (uint32_t)(((long)n * p.ldw + k) * 2) : SK_OOB;
        // weights are read once per decode step by one CU: nt (aux 2) shortens issued -> landed
        // (MI355X_MICROARCH nt-weights); SHAI_SKINNY_NT=0 restores the default policy
        if (p.w_nt)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (sk_lds_void*)(sw + (w * 2 + j) * 8 * SK_BK), 16, off, 0, 0,
                                                   2);
        else
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (sk_lds_void*)(sw + (w * 2 + j) * 8 * SK_BK), 16, off, 0, 0,
                                                   0);
      }
    }
#pragma unroll
    for (int j = 0; j < XG; ++j) {
      const int r = xr + 32 * j, k = k0 + xc * 8;
      const uint32_t off = (r < p.M && k < p.K) ? (uint32_t)(((long)r * p.lda + k) * 2) : SK_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (sk_lds_void*)(sx + (32 * j + w * 8) * SK_BK), 16, off, 0, 0,
                                               0);
    }
  };

  float16_ acc[2][XG];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < XG; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[h][j][i] = 0.f;
  float ss[XG];  // folded RMSNorm: this lane's share of sum_k X[m, k]^2 (the 4 waves x 2 halves together
                 // read every X element of every step exactly once)
#pragma unroll
  for (int j = 0; j < XG; ++j) ss[j] = 0.f;
  const int fr = lane & 31, fh = lane >> 5;
  const int ch = 2 * w + fh;  // this lane's 8-element chunk of the step's K range
#pragma unroll
  for (int i = 0; i < G::STAGES - 1; ++i)
    if (i < nk) stage(i, i);
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    sk_wait_upto<G::PER, G::STAGES - 2>(min(G::STAGES - 2, nk - 1 - kt));
    __builtin_amdgcn_s_barrier();
    if (kt + G::STAGES - 1 < nk) {
      const int nb = buf == 0 ? G::STAGES - 1 : buf - 1;  // buffer of step kt-1: every wave is past it
      stage(nb, kt + G::STAGES - 1);
    }
    const bf16_t* sw = sk_smem + buf * G::STAGE_ELEMS;
    const bf16_t* sx = sw + G::W_ELEMS;
    bf16x8s w0, w1;
    if constexpr (F8) {
      const char* swb = reinterpret_cast<const char*>(sw);
      w0 = sk_fp8x8(reinterpret_cast<const bf16_t*>(swb + sk_f8_off(fr, ch)));
      w1 = sk_fp8x8(reinterpret_cast<const bf16_t*>(swb + sk_f8_off(32 + fr, ch)));
    } else {
      w0 = *reinterpret_cast<const bf16x8s*>(sw + sk_swz(fr, ch));
      w1 = *reinterpret_cast<const bf16x8s*>(sw + sk_swz(32 + fr, ch));
    }
#pragma unroll
    for (int j = 0; j < XG; ++j) {
      const bf16x8s xf = *reinterpret_cast<const bf16x8s*>(sx + sk_swz(32 * j + fr, ch));
      acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, xf, acc[0][j], 0, 0, 0);
      acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, xf, acc[1][j], 0, 0, 0);
      if constexpr (RMS) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = (float)xf[e];
          ss[j] += f * f;
        }
      }
    }
    buf = buf == G::STAGES - 1 ? 0 : buf + 1;
  }
  if constexpr (RMS) {
#pragma unroll
    for (int j = 0; j < XG; ++j) ss_red[w][64 * j + lane] = ss[j];
  }

  // ---- cross-wave reduction through LDS (the stage ring is dead), 16-byte granules: wave w stores its partial tile
  // m-major, red[w][m][n] at a row pitch of SK_RP4 floats (16 B of bank skew per m row: conflict-free
  // ds_write_b128 / ds_read_b128), each lane's 4 consecutive-n accumulators (registers 4q .. 4q + 3: n = 8q + 4fh
  // + 0..3 of its 32-row half, m = 32j + fr) as ONE float4; a thread then owns output quads (m, 4 consecutive n) and
  // sums the 4 waves' float4s in wave order -- 4x fewer LDS instructions than element-wise, the epilogue / partial
  // stores 8-16 B per lane (gpurun_out/r6m_decode_lab2.log: the element-wise reduction + 4-B stores cost 2.4-3.9 us
  // per launch over the streaming loop).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float* red = reinterpret_cast<float*>(sk_smem);
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < XG; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = 32 * h + 8 * q + 4 * fh, m = 32 * j + fr;
        SHAI_DASSERT((w * MB + m) * SK_RP4 + n + 4 <= (int)(G::LDS / 4));
        *reinterpret_cast<float4_*>(red + (w * MB + m) * SK_RP4 + n) =
            float4_{acc[h][j][4 * q], acc[h][j][4 * q + 1], acc[h][j][4 * q + 2], acc[h][j][4 * q + 3]};
      }
  __syncthreads();
  auto row_ss = [&](int m) {
    const int j = m >> 5, r = m & 31;
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < SK_WAVES; ++q) t += ss_red[q][64 * j + r] + ss_red[q][64 * j + 32 + r];
    return t;
  };
  if constexpr (RMS) {
    if (KG == 1 && tid < MB) rstd_s[tid] = rsqrtf(row_ss(tid) / p.K + p.rms_eps);
    __syncthreads();
  }
  constexpr int QPT = MB * 16 / 256;  // output quads (m, 4 consecutive n) per thread
  // quad it of this thread: qd = tid + 256 it, m = qd >> 4, n = 4 (qd & 15); v = sum over waves in wave order,
  // times the fp8 row scale (per n) and, unsplit, the folded RMSNorm's rstd[m]
  auto qsum = [&](int it, float v[4]) {
    const int qd = tid + 256 * it, m = qd >> 4, n = 4 * (qd & 15);
    float4_ a = float4_{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < SK_WAVES; ++q) a += *reinterpret_cast<const float4_*>(red + (q * MB + m) * SK_RP4 + n);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = a[e];
      if constexpr (F8) v[e] *= (n0 + n + e < p.N) ? p.w_scale[n0 + n + e] : 0.f;
      if constexpr (RMS) {
        if (KG == 1) v[e] *= rstd_s[m];
      }
    }
  };
  // fused epilogue of quad (m, n): 4 consecutive outputs (2 GLU pairs) with 8-B stores where the quad is whole
  auto quad_out = [&](int m, int n, float v[4]) {
    if (m >= p.M || n0 + n >= p.N) return;
    if (n0 + n + 3 < p.N) {
      epilogue4<GLU, ACT>(p, p.C, p.residual, m, n0 + n, v);
    } else if constexpr (GLU) {
      for (int e = 0; e < 4 && n0 + n + e + 1 < p.N; e += 2) sk_store<GLU, ACT>(p, n0 + n + e, m, v[e], v[e + 1]);
    } else {
      for (int e = 0; e < 4; ++e) sk_store<GLU, ACT>(p, n0 + n + e, m, v[e], 0.f);
    }
  };
  if (KG == 1) {
#pragma unroll
    for (int it = 0; it < QPT; ++it) {
      float v[4];
      qsum(it, v);
      const int qd = tid + 256 * it;
      quad_out(qd >> 4, 4 * (qd & 15), v);
    }
    return;
  }
  if (cnt != nullptr) {
    // ---- split-K fixed up in this launch (no reduce kernel): every K group writes its 64 x MB partial slab
    // (+ MB row sums of squares) write-through (sc1, 16 B per lane), drains (vmcnt 0 in every wave), joins the
    // workgroup barrier, then one lane takes a ticket (relaxed agent-scope atomic on this launch's own ticket
    // slice, sk_tickets); the workgroup that draws KG-1 re-arms the ticket and reduces the KG slabs with sc1
    // loads before the fused epilogue.
    // (MI355X_MICROARCH / hip guide "Projection GEMM at M = 256" item 2, write-through form.)
    // Slab layout: element m * 64 + n, i.e. float4 qd of this thread at byte 16 qd.
    constexpr int SLAB = 64 * MB + MB;
    const __amdgpu_buffer_rsrc_t rws = sk_rsrc(ws, 0x7fffffffu);
    const uint32_t tile_base = (uint32_t)((long)tile * KG * SLAB * 4);
    const uint32_t my_base = tile_base + (uint32_t)(kg * SLAB * 4);
    float part[QPT][4];
#pragma unroll
    for (int it = 0; it < QPT; ++it) {
      qsum(it, part[it]);
      sk_store_wt4(rws, my_base + (tid + 256 * it) * 16, part[it]);
    }
    float ssv = 0.f;
    if constexpr (RMS) {
      if (tid < MB) {
        ssv = row_ss(tid);
        sk_store_wt(rws, my_base + (64 * MB + tid) * 4, ssv);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ unsigned sk_last;
    if (tid == 0) {
      // The hand-off follows the write-through publish form (cdna_hip_programming.md Guideline 16, R1 with
      // sc1 consumer loads): every slab byte is stored sc1 by its writing wave, EVERY wave drains vmcnt(0)
      // before the workgroup barrier above, the signal is an agent-scope atomic, and the last arriver reads
      // the slabs ONLY with sc1 loads into registers (sk_load_wt*) -- no other load of this launch touches
      // bytes another workgroup wrote.  So the ticket is relaxed and the acquire is a wavefront-scope fence
      // (no instruction: it only keeps the compiler from hoisting the slab loads above the ticket).  An
      // agent-scope acq_rel here (buffer_wbl2 + buffer_inv of the XCD's L2) measured -7 % Mistral decode.
      const unsigned old = __hip_atomic_fetch_add(&cnt[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      sk_last = old == (unsigned)(KG - 1);
    }
    __syncthreads();
    if (sk_last == 0u) return;
    if (tid == 0) __hip_atomic_store(&cnt[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // sum the KG slabs in K-group order (this group's own slab from registers), so the result does not
    // depend on which group arrived last: four slabs at a time with every load issued before the first add
    // (slots past KG, and this group's own slot, re-read this group's slab and substitute / drop it)
    float own[QPT][4], sum[QPT][4], own_ss = ssv;
#pragma unroll
    for (int it = 0; it < QPT; ++it)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        own[it][e] = part[it][e];
        sum[it][e] = 0.f;
      }
    ssv = 0.f;
    for (int u0 = 0; u0 < KG; u0 += 4) {
      float4_ t[4][QPT];
      float ts[4];
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) {
        const int q = u0 + uu < KG ? u0 + uu : kg;
        const uint32_t b = tile_base + (uint32_t)(q * SLAB * 4);
#pragma unroll
        for (int it = 0; it < QPT; ++it) t[uu][it] = sk_load_wt4(rws, b + (tid + 256 * it) * 16);
        ts[uu] = 0.f;
        if constexpr (RMS) ts[uu] = sk_load_wt(rws, b + (64 * MB + (tid & (MB - 1))) * 4);
      }
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) {
        const int q = u0 + uu;
        if (q < KG) {
          const bool mine = q == kg;
#pragma unroll
          for (int it = 0; it < QPT; ++it)
#pragma unroll
            for (int e = 0; e < 4; ++e) sum[it][e] += mine ? own[it][e] : t[uu][it][e];
          ssv += mine ? own_ss : ts[uu];
        }
      }
    }
    if constexpr (RMS) {
      if (tid < MB) rstd_s[tid] = rsqrtf(ssv / p.K + p.rms_eps);
      __syncthreads();
    }
#pragma unroll
    for (int it = 0; it < QPT; ++it) {
      const int qd = tid + 256 * it, m = qd >> 4;
      if constexpr (RMS) {
#pragma unroll
        for (int e = 0; e < 4; ++e) sum[it][e] *= rstd_s[m];
      }
      quad_out(m, 4 * (qd & 15), sum[it]);
    }
    return;
  }
  if constexpr (RMS) {  // row sum-of-squares partials for the fold (one tile per K group writes them)
    if (tile == 0 && tid < p.M) ws[(long)KG * p.M * p.N + (long)kg * p.M + tid] = row_ss(tid);
  }
  // ---- split-K over workgroups: fp32 partials [kg][M][N]; launch_splitk_epilogue (or the decode attention's QKV
  // fold) folds them.  16 B per lane where the quad is whole and N keeps rows 16-B aligned.
  float* part = ws + (long)kg * p.M * p.N;
#pragma unroll
  for (int it = 0; it < QPT; ++it) {
    float v[4];
    qsum(it, v);
    const int qd = tid + 256 * it, m = qd >> 4, n = n0 + 4 * (qd & 15);
    if (m >= p.M || n >= p.N) continue;
    if (n + 3 < p.N && (p.N & 3) == 0) {
      *reinterpret_cast<float4_*>(part + (long)m * p.N + n) = float4_{v[0], v[1], v[2], v[3]};
    } else {
      for (int e = 0; e < 4 && n + e < p.N; ++e) part[(long)m * p.N + n + e] = v[e];
    }
  }
}

// fp8 (e4m3) rows x per-row scale -> bf16 (prefill-shaped problems run the bf16 GEMMs on it)
__global__ void __launch_bounds__(256) dequant_fp8_rows_kernel(const uint8_t* __restrict__ w8,
                                                               const float* __restrict__ scale,
                                                               bf16_t* __restrict__ out, long total8, int K8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total8; i += (long)gridDim.x * blockDim.x) {
    const float sc = scale[i / K8];
    const uint2_ v = reinterpret_cast<const uint2_*>(w8)[i];
    float f[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)v[h], false);
      const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)v[h], true);
      f[4 * h + 0] = lo[0] * sc;
      f[4 * h + 1] = lo[1] * sc;
      f[4 * h + 2] = hi[0] * sc;
      f[4 * h + 3] = hi[1] * sc;
    }
    reinterpret_cast<uint4_*>(out)[i] = pack8(f);
  }
}

void launch_dequant_fp8_rows(const uint8_t* w8, const float* scale, bf16_t* out, long N, int K, hipStream_t s) {
  const long total8 = N * (long)K / 8;
  long blocks = (total8 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  dequant_fp8_rows_kernel<<<(int)blocks, 256, 0, s>>>(w8, scale, out, total8, K / 8);
}

// ---------------------------------------------------------------------------- host side
bool skinny_supported(const GemmArgs& a) {
  return !a.conv && (a.batch <= 1) && a.w_slice_rows == 0 && a.M >= 1 && a.M <= 64 && a.K % 8 == 0 && a.N % 2 == 0 &&
         a.bias2d == nullptr && a.gate == nullptr && a.in_scale == nullptr && a.row_mr == nullptr && (a.lda % 8) == 0 &&
         (a.ldw % (a.w_scale ? 16 : 8)) == 0 && (long)a.N * a.ldw * 2 < 0x7fffffffL;
}

// K groups: enough workgroups for ~2 per CU, each group >= 2 pipeline depths of K steps.
int skinny_kgroups(const GemmArgs& a) {
  const int stages = a.M <= 32 ? SkGeom<32>::STAGES : SkGeom<64>::STAGES;
  const int tiles = (a.N + SK_BN - 1) / SK_BN, ksteps = (a.K + SK_BK - 1) / SK_BK;
  int kg = 1;
  while (tiles * kg < 512 && ksteps / (kg * 2) >= stages) kg *= 2;
  return kg;
}

size_t skinny_workspace_bytes_kg(const GemmArgs& a, int kg) {
  if (kg <= 1) return 0;
  const size_t fold = (size_t)kg * a.M * a.N + (a.rms ? (size_t)kg * a.M : 0);    // [kg][M][N] + row sums
  const int MB = a.M <= 32 ? 32 : 64;
  const size_t fix = (size_t)((a.N + SK_BN - 1) / SK_BN) * kg * (64 * MB + MB);  // [tile][kg] slabs
  return (fold > fix ? fold : fix) * sizeof(float);
}

size_t skinny_workspace_bytes(const GemmArgs& a) { return skinny_workspace_bytes_kg(a, skinny_kgroups(a)); }

int skinny_max_kgroups(const GemmArgs& a) {
  const int ksteps = (a.K + SK_BK - 1) / SK_BK;
  int kg = 1;
  while (kg < 16 && ksteps / (kg * 2) >= 2) kg *= 2;
  return kg;
}

// Arrival tickets of the in-kernel split-K fixup.  One pool per device (kSkPool tickets, zeroed once, outside
// any capture); every launch counts arrivals in a slice of it that no launch able to run at the same time
// shares: a launch being captured into a HIP graph takes a fresh slice from a bump allocator (the graph keeps
// it for its lifetime: replays of one graph are serialised by its own buffers), an eager launch uses the
// slice owned by its stream.  The last arriver re-arms its ticket, so a slice serves every later launch on
// the same stream / replay of the same graph.  No slice (pool not yet allocated while capturing, or
// exhausted) -> the separate fold kernel, which needs no tickets.
constexpr int kSkTickets = 4096;            // max tiles of one launch (and the per-stream slice)
constexpr size_t kSkPool = size_t(1) << 24;  // 16 M tickets = 64 MB per device

struct SkTicketPool {
  unsigned* base = nullptr;
  size_t next = 0;
  std::map<hipStream_t, unsigned*> per_stream;
};

static unsigned* sk_tickets(hipStream_t s, int ntiles) {
  static std::mutex mu;
  static SkTicketPool pools[64];
  int dev = 0;
  if (ntiles > kSkTickets || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess) return nullptr;
  const bool capturing = cs != hipStreamCaptureStatusNone;
  std::lock_guard<std::mutex> lock(mu);
  SkTicketPool& P = pools[dev];
  if (P.base == nullptr) {
    if (capturing) return nullptr;  // never allocate inside a graph capture
    unsigned* p = nullptr;
    if (hipMalloc(&p, kSkPool * sizeof(unsigned)) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, kSkPool * sizeof(unsigned)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(p);
      return nullptr;
    }
    P.base = p;
  }
  if (!capturing) {
    auto it = P.per_stream.find(s);
    if (it != P.per_stream.end()) return it->second;
  }
  const size_t want = capturing ? (size_t)ntiles : (size_t)kSkTickets;
  if (P.next + want > kSkPool) return nullptr;
  unsigned* slice = P.base + P.next;
  P.next += (want + 63) & ~size_t(63);
  if (!capturing) P.per_stream[s] = slice;
  return slice;
}

unsigned* skinny_ticket_slice(hipStream_t s, int ntiles) { return sk_tickets(s, ntiles); }

template <int MB, bool F8>
static void launch_skinny_mb(const GemmArgs& a, float* ws, int kg, unsigned* cnt, hipStream_t s) {
  const int ksteps = (a.K + SK_BK - 1) / SK_BK;
  const int kg_steps = (ksteps + kg - 1) / kg;
  dim3 grid((a.N + SK_BN - 1) / SK_BN, kg), block(SK_WAVES * 64);
  const size_t lds = SkGeom<MB, F8>::LDS;
#define SK(G, A)                                                                                          \
  do {                                                                                                    \
    if (a.rms) skinny_gemm_kernel<MB, G, A, true, F8><<<grid, block, lds, s>>>(a, ws, kg_steps, cnt);  \
    else skinny_gemm_kernel<MB, G, A, false, F8><<<grid, block, lds, s>>>(a, ws, kg_steps, cnt);       \
  } while (0)
#define SK_ACT(G)                                      \
  switch (a.act) {                                     \
    case ACT_SILU: SK(G, ACT_SILU); break;             \
    case ACT_GELU: SK(G, ACT_GELU); break;             \
    case ACT_GELU_TANH: SK(G, ACT_GELU_TANH); break;   \
    case ACT_QUICK_GELU: SK(G, ACT_QUICK_GELU); break; \
    case ACT_RELU: SK(G, ACT_RELU); break;             \
    default: SK(G, ACT_NONE); break;                   \
  }
  if (a.glu) {
    SK_ACT(true)
  } else {
    SK_ACT(false)
  }
#undef SK_ACT
#undef SK
}

// kg K groups (split-K over workgroups; needs ws of skinny_workspace_bytes_kg, else kg = 1)
void launch_skinny_kg(const GemmArgs& a_in, float* ws, int kg, hipStream_t s, bool fixup, bool fold) {
  static const int nt = [] {
    const char* e = getenv("SHAI_SKINNY_NT");
    return e ? atoi(e) : 1;
  }();
  GemmArgs a = a_in;
  a.w_nt = nt;
  const int ksteps = (a.K + SK_BK - 1) / SK_BK;
  if (ws == nullptr || kg < 1) kg = 1;
  if (kg > ksteps) kg = ksteps;
  // split-K: fixed up inside the launch when asked for and tickets are available, else a separate fold
  unsigned* cnt = nullptr;
  if (kg > 1 && fixup) cnt = sk_tickets(s, (a.N + SK_BN - 1) / SK_BN);
  if (a.w_scale) {
    if (a.M <= 32) launch_skinny_mb<32, true>(a, ws, kg, cnt, s);
    else launch_skinny_mb<64, true>(a, ws, kg, cnt, s);
  } else {
    if (a.M <= 32) launch_skinny_mb<32, false>(a, ws, kg, cnt, s);
    else launch_skinny_mb<64, false>(a, ws, kg, cnt, s);
  }
  if (kg > 1 && cnt == nullptr && fold) launch_splitk_epilogue(a, ws, kg, s);
}

void launch_skinny(const GemmArgs& a, float* ws, hipStream_t s) {
  launch_skinny_kg(a, ws, ws != nullptr ? skinny_kgroups(a) : 1, s);
}

}  // namespace shai
