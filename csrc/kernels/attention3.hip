// flash64 with LDS-DMA K/V staging (`launch_flash64_dma`, production for D = 64): the register-staged K/V pipeline of
// flash64 (attention.hip) holds 16 VGPRs of next-tile K/V plus the ds_write pass; staging the tiles with
// `buffer_load ... lds` (source-side swizzle, lane-linear LDS image) frees them, and the softmax computes P in
// chunks of 8 exponentials instead of a 32-float buffer, so the kernel can aim at 4 waves per SIMD (128 VGPRs)
// instead of 3 (168): more co-resident waves to overlap one wave's MFMAs with another's softmax, which is what
// bounds D = 64 attention (VALU issue + latency, profiles/pmc_round3.md: 37 % MFMA busy).  Measured (attention lab,
// round 4): at 3 waves / SIMD (150 VGPRs) 906 vs 821 TF/s at the SD2.1 64x64 shape, 616 vs 557 at 32x32; forcing 4
// waves spills (23 VGPRs) and halves the rate, so production runs the 3-wave build (the 4-wave one is retired).
//
// flash64x2 (below) doubles the queries per wave; launch_flash64 picks it when the launch has >= 1024 of its
// 256-query workgroups (the SD2.1 batch-64 shapes), the 128-query kernel for smaller grids where the x2 grid's tail
// costs more than it gains.  Round 5 attention lab (tools/gemm_lab/attn_lab.cpp, this file built with
// -mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize as csrc/build.py does): B64 H5 S4096 1330 us (1033 TF/s) vs
// 1378 us for the 128-query kernel and 1430 us before the flags; B64 H10 S1024 202 vs 225 us.  A variant that
// software-pipelines the two groups half a tile apart (QK / PV of one group beside the other's exponentials, no
// branch on the fast path) measured 1433-1491 us: hipcc kept its LDS reads just in time (a lgkmcnt(0) before every
// MFMA) at 246 VGPRs, so it was dropped.
#include "common.h"
#include "launchers.h"

#include <type_traits>

namespace shai {

typedef __bf16 f3bf16x8 __attribute__((ext_vector_type(8)));
typedef short f3s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void f3_lds_void;

__device__ __forceinline__ int f3_kswz(int row, int ch) { return row * 64 + ((ch ^ ((row >> 1) & 7)) << 3); }
__device__ __forceinline__ int f3_vswz(int row, int ch) { return row * 64 + ((ch ^ (((row >> 1) & 1) << 2)) << 3); }

template <int OCC, bool CAUSAL>
__global__ void __launch_bounds__(256, OCC) flash64_dma_kernel(const AttnArgs p) {
  constexpr int D = 64, KT = 64, NS = 4, ND = 2;
  constexpr float kSumThr = 256.f;
  constexpr float kL2e = 1.4426950408889634f;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  // stage s: K tile at smem + s * 2 * KT * D, V tile right after it

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 31, fh = lane >> 5;
  const int b = blockIdx.z, hq = blockIdx.y;
  const int hk = hq / (p.Hq / p.Hkv);
  const int q_len = p.q_lens ? p.q_lens[b] : p.Sq;
  const int kv_len = p.kv_lens ? p.kv_lens[b] : p.Skv;
  const int c_off = p.q_lens ? kv_len - q_len : p.causal_offset;
  if ((int)blockIdx.x * 128 >= q_len) return;
  const int q0 = blockIdx.x * 128;
  const int qi = q0 + wid * 32 + fr;
  const float sl2 = p.scale * kL2e;

  const bf16_t* kbase = p.k + (long)b * p.k_bs + (long)hk * D;
  const bf16_t* vbase = p.v + (long)b * p.v_bs + (long)hk * D;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(kbase), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(vbase), (short)0, 0x7fffffff, 0x00020000);
  int kv_end = kv_len;
  if (CAUSAL) kv_end = min(kv_end, q0 + 127 + c_off + 1);
  const int ntiles = kv_end > 0 ? (kv_end + KT - 1) / KT : 0;
  // DMA: wave wid moves K rows 16 wid + 8 i + (lane >> 3) (i < 2) and the same V rows; lane position lane & 7
  // of the 128-B row receives source chunk (pos ^ swizzle(row))
  const int drow = wid * 16 + (lane >> 3), dpos = lane & 7;
  const int kch0 = dpos ^ ((drow >> 1) & 7), kch1 = dpos ^ (((drow + 8) >> 1) & 7);
  const int vch0 = dpos ^ (((drow >> 1) & 1) << 2), vch1 = dpos ^ ((((drow + 8) >> 1) & 1) << 2);
  auto dma = [&](int stage, int t) {
    bf16_t* ks = smem + stage * 2 * KT * D;
    bf16_t* vs = ks + KT * D;
    const int key = t * KT + drow;
    const uint32_t ok0 = key < kv_len ? 0u : 0x80000000u, ok1 = key + 8 < kv_len ? 0u : 0x80000000u;
    const uint32_t r0 = (uint32_t)((long)key * p.k_ts * 2), r1 = (uint32_t)((long)(key + 8) * p.k_ts * 2);
    const uint32_t v0 = (uint32_t)((long)key * p.v_ts * 2), v1 = (uint32_t)((long)(key + 8) * p.v_ts * 2);
    // debug: a valid key's byte offset fits the 31-bit buffer range (no wrap into the OOB sentinel), ring slot
    SHAI_DASSERT(ok0 != 0u || ((long)key * p.k_ts * 2 + 128 < 0x80000000L && (long)key * p.v_ts * 2 + 128 < 0x80000000L));
    SHAI_DASSERT(ok1 != 0u || ((long)(key + 8) * p.k_ts * 2 + 128 < 0x80000000L));
    SHAI_DASSERT(stage == 0 || stage == 1);  // two K/V stages of LDS (launchers size 2 x 2 x 64 x 64)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (f3_lds_void*)(ks + (wid * 16) * D), 16, (r0 + kch0 * 16) | ok0, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (f3_lds_void*)(ks + (wid * 16 + 8) * D), 16, (r1 + kch1 * 16) | ok1, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (f3_lds_void*)(vs + (wid * 16) * D), 16, (v0 + vch0 * 16) | ok0, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (f3_lds_void*)(vs + (wid * 16 + 8) * D), 16, (v1 + vch1 * 16) | ok1, 0, 0, 0);
  };
  if (ntiles > 0) dma(0, 0);

  f3bf16x8 qf[NS];
  {
    const bf16_t* qp = p.q + (p.q_start ? (long)p.q_start[b] * p.q_ts : (long)b * p.q_bs) +
                        (long)min(qi, q_len - 1) * p.q_ts + (long)hq * D;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      uint4_ v = *reinterpret_cast<const uint4_*>(qp + 16 * s + 8 * fh);
      if (qi >= q_len) v = uint4_{0u, 0u, 0u, 0u};
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= sl2;
      qf[s] = __builtin_bit_cast(f3bf16x8, pack8(f));
    }
  }

  float16_ o[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  const f3bf16x8 a_one = __builtin_bit_cast(f3bf16x8, uint4_{lane < 32 ? 0x3F80u : 0u, 0u, 0u, 0u});
  f3bf16x8 b_negm = __builtin_bit_cast(f3bf16x8, uint4_{0u, 0u, 0u, 0u});

  const int g16 = lane >> 4, i16 = lane & 15;
  const int tq = i16 >> 2, tp = i16 & 3;
  int koff[NS], voff[ND];
#pragma unroll
  for (int s = 0; s < NS; ++s) koff[s] = f3_kswz(fr, 2 * s + fh);
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    const int col = d * 32 + 16 * (g16 & 1) + 4 * tp;
    voff[d] = f3_vswz(4 * fh + tq, col >> 3) + 4 * ((col >> 2) & 1);
  }

  float16_ sacc[2];
  f3bf16x8 pf[2][2];
  // P = exp2(acc (+ add)) in four chunks of 8 exponentials (no 32-float buffer); returns the lane's row sum
  auto expo = [&](float add, auto addt) {
    constexpr bool ADD = decltype(addt)::value;
    float ls4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) e[j] = __builtin_amdgcn_exp2f(ADD ? sacc[kb][8 * s + j] + add : sacc[kb][8 * s + j]);
        f3bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          ls4[j & 3] += e[j];
          v[j] = (__bf16)e[j];
        }
        pf[kb][s] = v;
      }
    return (ls4[0] + ls4[1]) + (ls4[2] + ls4[3]);
  };

  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    // tile t's DMA (this wave's part) landed; every wave past its reads of the other stage (tile t-1)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < ntiles) dma(cur ^ 1, t + 1);
    const bf16_t* ks = smem + cur * 2 * KT * D;
    const bf16_t* vs = ks + KT * D;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const float16_ z = {};
      sacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_one, b_negm, z, 0, 0, 0);
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const f3bf16x8 kf = *reinterpret_cast<const f3bf16x8*>(ks + koff[s] + kb * 2048);
        sacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc[kb], 0, 0, 0);
      }
    }
    const int key0 = t * KT;
    if ((key0 + KT > kv_len) || (CAUSAL && key0 + KT - 1 > q0 + c_off)) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = key0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          const bool bad = key >= kv_len || (CAUSAL && key > qi + c_off);
          sacc[kb][r] = bad ? -INFINITY : sacc[kb][r];
        }
    }
    float ls = 0.f;
    bool slow = __any(m_run == -INFINITY);
    if (!slow) {
      ls = expo(0.f, std::false_type{});
      slow = __any(!(ls <= kSumThr));
    }
    if (slow) {
      float m4[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) m4[r & 3] = fmaxf(m4[r & 3], sacc[kb][r]);
      const float mb = m_run == -INFINITY ? 0.f : m_run;
      float mloc = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64)) + mb;
      // round the max up onto the bf16 grid (it enters the -m MFMA as a bf16 operand exactly)
      uint32_t u = __float_as_uint(fmaxf(m_run, mloc));
      if ((u & 0xffffu) != 0u && u != 0xff800000u) u = (u & 0x80000000u) ? (u & 0xffff0000u) : ((u + 0x10000u) & 0xffff0000u);
      const float m_new = __uint_as_float(u);
      const float m_use = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[d][r] *= alpha;
      l_run *= alpha;
      const float shift = mb - m_use;
      m_run = m_new;
      const uint32_t nb = __float_as_uint(-(m_run == -INFINITY ? 0.f : m_run)) >> 16;
      b_negm = __builtin_bit_cast(f3bf16x8, uint4_{lane < 32 ? nb : 0u, 0u, 0u, 0u});
      ls = expo(shift, std::true_type{});
    }
    l_run += ls;
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16_t* a0 = vs + voff[d] + kb * 2048 + s * 1024;
          const f3s4v t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) f3s4v*)(a0));
          const f3s4v t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) f3s4v*)(a0 + 512));
          short8 vv;
          vv[0] = t0[0]; vv[1] = t0[1]; vv[2] = t0[2]; vv[3] = t0[3];
          vv[4] = t1[0]; vv[5] = t1[1]; vv[6] = t1[2]; vv[7] = t1[3];
          o[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(f3bf16x8, vv), pf[kb][s], o[d], 0, 0, 0);
        }
    // every wave's reads of this stage retire before the next iteration's barrier (restaged after it)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qi < q_len) {
    bf16_t* op = p.o + (p.q_start ? (long)p.q_start[b] * p.o_ts : (long)b * p.o_bs) + (long)qi * p.o_ts +
                 (long)hq * D;
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = d * 32 + 8 * g + 4 * fh;
        uint2_ w;
        w[0] = pack2(o[d][4 * g] * inv, o[d][4 * g + 1] * inv);
        w[1] = pack2(o[d][4 * g + 2] * inv, o[d][4 * g + 3] * inv);
        *reinterpret_cast<uint2_*>(op + dd) = w;
      }
  }
}

// flash64x2: the same K/V pipeline with TWO groups of 32 queries per wave (64 per wave, 256 per workgroup).  The two
// groups' chains are independent: group B's score MFMAs are in the matrix pipe while group A's exponentials run on the
// VALU, and A's P.V MFMAs beside B's exponentials (each V fragment read once for both) -- the overlap a single
// 32-query chain (QK -> softmax -> PV, each waiting on the last) can only get from other waves.  The softmax fast path
// is branch-free (the mask and the lazy-max rescale run after it, on a wave-uniform branch), which keeps each pair in
// one basic block: round-5 lab, same box, 1397 vs 1443 us at B64 H5 S4096 and 209 vs 225 us at B64 H10 S1024 for
// the branchy order (QK both -> softmax A -> PV A -> softmax B -> PV B).  2 waves / SIMD (<= 256 registers).
template <bool CAUSAL>
__global__ void __launch_bounds__(256, 2) flash64x2_kernel(const AttnArgs p) {
  constexpr int D = 64, KT = 64, NS = 4, ND = 2, G = 2;
  constexpr float kSumThr = 256.f;
  constexpr float kL2e = 1.4426950408889634f;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 31, fh = lane >> 5;
  const int b = blockIdx.z, hq = blockIdx.y;
  const int hk = hq / (p.Hq / p.Hkv);
  const int q_len = p.q_lens ? p.q_lens[b] : p.Sq;
  const int kv_len = p.kv_lens ? p.kv_lens[b] : p.Skv;
  const int c_off = p.q_lens ? kv_len - q_len : p.causal_offset;
  if ((int)blockIdx.x * 256 >= q_len) return;
  const int q0 = blockIdx.x * 256;
  int qi[G];
#pragma unroll
  for (int g = 0; g < G; ++g) qi[g] = q0 + wid * 64 + 32 * g + fr;
  const float sl2 = p.scale * kL2e;

  const bf16_t* kbase = p.k + (long)b * p.k_bs + (long)hk * D;
  const bf16_t* vbase = p.v + (long)b * p.v_bs + (long)hk * D;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(kbase), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(vbase), (short)0, 0x7fffffff, 0x00020000);
  int kv_end = kv_len;
  if (CAUSAL) kv_end = min(kv_end, q0 + 255 + c_off + 1);
  const int ntiles = kv_end > 0 ? (kv_end + KT - 1) / KT : 0;
  const int drow = wid * 16 + (lane >> 3), dpos = lane & 7;
  const int kch0 = dpos ^ ((drow >> 1) & 7), kch1 = dpos ^ (((drow + 8) >> 1) & 7);
  const int vch0 = dpos ^ (((drow >> 1) & 1) << 2), vch1 = dpos ^ ((((drow + 8) >> 1) & 1) << 2);
  auto dma = [&](int stage, int t) {
    bf16_t* ks = smem + stage * 2 * KT * D;
    bf16_t* vs = ks + KT * D;
    const int key = t * KT + drow;
    const uint32_t ok0 = key < kv_len ? 0u : 0x80000000u, ok1 = key + 8 < kv_len ? 0u : 0x80000000u;
    const uint32_t r0 = (uint32_t)((long)key * p.k_ts * 2), r1 = (uint32_t)((long)(key + 8) * p.k_ts * 2);
    const uint32_t v0 = (uint32_t)((long)key * p.v_ts * 2), v1 = (uint32_t)((long)(key + 8) * p.v_ts * 2);
    // debug: a valid key's byte offset fits the 31-bit buffer range (no wrap into the OOB sentinel), ring slot
    SHAI_DASSERT(ok0 != 0u || ((long)key * p.k_ts * 2 + 128 < 0x80000000L && (long)key * p.v_ts * 2 + 128 < 0x80000000L));
    SHAI_DASSERT(ok1 != 0u || ((long)(key + 8) * p.k_ts * 2 + 128 < 0x80000000L));
    SHAI_DASSERT(stage == 0 || stage == 1);  // two K/V stages of LDS (launchers size 2 x 2 x 64 x 64)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (f3_lds_void*)(ks + (wid * 16) * D), 16, (r0 + kch0 * 16) | ok0, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (f3_lds_void*)(ks + (wid * 16 + 8) * D), 16, (r1 + kch1 * 16) | ok1, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (f3_lds_void*)(vs + (wid * 16) * D), 16, (v0 + vch0 * 16) | ok0, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (f3_lds_void*)(vs + (wid * 16 + 8) * D), 16, (v1 + vch1 * 16) | ok1, 0, 0, 0);
  };
  if (ntiles > 0) dma(0, 0);

  f3bf16x8 qf[G][NS];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const bf16_t* qp = p.q + (p.q_start ? (long)p.q_start[b] * p.q_ts : (long)b * p.q_bs) +
                        (long)min(qi[g], q_len - 1) * p.q_ts + (long)hq * D;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      uint4_ v = *reinterpret_cast<const uint4_*>(qp + 16 * s + 8 * fh);
      if (qi[g] >= q_len) v = uint4_{0u, 0u, 0u, 0u};
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= sl2;
      qf[g][s] = __builtin_bit_cast(f3bf16x8, pack8(f));
    }
  }

  float16_ o[G][ND];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[g][d][r] = 0.f;
  float m_run[G], l_run[G];
  f3bf16x8 b_negm[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m_run[g] = -INFINITY;
    l_run[g] = 0.f;
    b_negm[g] = __builtin_bit_cast(f3bf16x8, uint4_{0u, 0u, 0u, 0u});
  }
  const f3bf16x8 a_one = __builtin_bit_cast(f3bf16x8, uint4_{lane < 32 ? 0x3F80u : 0u, 0u, 0u, 0u});

  const int g16 = lane >> 4, i16 = lane & 15;
  const int tq = i16 >> 2, tp = i16 & 3;
  int koff[NS], voff[ND];
#pragma unroll
  for (int s = 0; s < NS; ++s) koff[s] = f3_kswz(fr, 2 * s + fh);
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    const int col = d * 32 + 16 * (g16 & 1) + 4 * tp;
    voff[d] = f3_vswz(4 * fh + tq, col >> 3) + 4 * ((col >> 2) & 1);
  }

  float16_ sacc[G][2];
  f3bf16x8 pf[G][2][2];
  auto expo = [&](int g, float add, auto addt) {
    constexpr bool ADD = decltype(addt)::value;
    float ls4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          e[j] = __builtin_amdgcn_exp2f(ADD ? sacc[g][kb][8 * s + j] + add : sacc[g][kb][8 * s + j]);
        f3bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          ls4[j & 3] += e[j];
          v[j] = (__bf16)e[j];
        }
        pf[g][kb][s] = v;
      }
    return (ls4[0] + ls4[1]) + (ls4[2] + ls4[3]);
  };
  // the slow path of group g's softmax for the tile at key0 (lazy max: rescale only when the tile's row sum would
  // exceed 2^8), after a branch-free fast path (ls_fast, pf[g] already computed): masking and the rescale only here,
  // so the fast path's exponentials share a basic block with the other group's MFMAs and the scheduler can
  // interleave them
  auto check = [&](int g, int key0, float ls_fast) {
    const bool mask = (key0 + KT > kv_len) || (CAUSAL && key0 + KT - 1 > q0 + wid * 64 + 32 * g + c_off);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) asm volatile("" ::"v"(pf[g][kb][s2]));
    asm volatile("" ::"v"(ls_fast));
    const uint64_t slow_lanes = __ballot(m_run[g] == -INFINITY) | __ballot(!(ls_fast <= kSumThr));
    float ls = ls_fast;
    if (mask | (slow_lanes != 0)) {
      if (mask) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = key0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
            const bool bad = key >= kv_len || (CAUSAL && key > qi[g] + c_off);
            sacc[g][kb][r] = bad ? -INFINITY : sacc[g][kb][r];
          }
      }
      float m4[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) m4[r & 3] = fmaxf(m4[r & 3], sacc[g][kb][r]);
      const float mb = m_run[g] == -INFINITY ? 0.f : m_run[g];
      float mloc = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64)) + mb;
      uint32_t u = __float_as_uint(fmaxf(m_run[g], mloc));
      if ((u & 0xffffu) != 0u && u != 0xff800000u) u = (u & 0x80000000u) ? (u & 0xffff0000u) : ((u + 0x10000u) & 0xffff0000u);
      const float m_new = __uint_as_float(u);
      const float m_use = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f(m_run[g] - m_use);
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[g][d][r] *= alpha;
      l_run[g] *= alpha;
      const float shift = mb - m_use;
      m_run[g] = m_new;
      const uint32_t nb = __float_as_uint(-(m_run[g] == -INFINITY ? 0.f : m_run[g])) >> 16;
      b_negm[g] = __builtin_bit_cast(f3bf16x8, uint4_{lane < 32 ? nb : 0u, 0u, 0u, 0u});
      ls = expo(g, shift, std::true_type{});
    }
    l_run[g] += ls;
  };
  auto qk1 = [&](int g, const bf16_t* ks) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const float16_ z = {};
      sacc[g][kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_one, b_negm[g], z, 0, 0, 0);
#pragma unroll
      for (int s2 = 0; s2 < NS; ++s2) {
        const f3bf16x8 kf = *reinterpret_cast<const f3bf16x8*>(ks + koff[s2] + kb * 2048);
        sacc[g][kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[g][s2], sacc[g][kb], 0, 0, 0);
      }
    }
  };

  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < ntiles) dma(cur ^ 1, t + 1);
    const bf16_t* ks = smem + cur * 2 * KT * D;
    const bf16_t* vs = ks + KT * D;
    {
      // QK_A; then QK_B beside A's exponentials; A's P.V beside B's exponentials; B's P.V
      const int key0 = t * KT;
      qk1(0, ks);
      qk1(1, ks);
      const float ls0 = expo(0, 0.f, std::false_type{});
      check(0, key0, ls0);
      f3bf16x8 vf[ND][2][2];
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const bf16_t* a0 = vs + voff[d] + kb * 2048 + s2 * 1024;
            const f3s4v t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) f3s4v*)(a0));
            const f3s4v t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) f3s4v*)(a0 + 512));
            vf[d][kb][s2] = __builtin_bit_cast(f3bf16x8, __builtin_shufflevector(t0, t1, 0, 1, 2, 3, 4, 5, 6, 7));
            o[0][d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[d][kb][s2], pf[0][kb][s2], o[0][d], 0, 0, 0);
          }
      const float ls1 = expo(1, 0.f, std::false_type{});
      check(1, key0, ls1);
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
            o[1][d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[d][kb][s2], pf[1][kb][s2], o[1][d], 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }

#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float l_tot = l_run[g] + __shfl_xor(l_run[g], 32, 64);
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    if (qi[g] < q_len) {
      bf16_t* op = p.o + (p.q_start ? (long)p.q_start[b] * p.o_ts : (long)b * p.o_bs) + (long)qi[g] * p.o_ts +
                   (long)hq * D;
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          const int dd = d * 32 + 8 * gg + 4 * fh;
          uint2_ w;
          w[0] = pack2(o[g][d][4 * gg] * inv, o[g][d][4 * gg + 1] * inv);
          w[1] = pack2(o[g][d][4 * gg + 2] * inv, o[g][d][4 * gg + 3] * inv);
          *reinterpret_cast<uint2_*>(op + dd) = w;
        }
    }
  }
}

void launch_flash64_x2(const AttnArgs& a, hipStream_t s) {
  dim3 grid((a.Sq + 255) / 256, a.Hq, a.B);
  const size_t lds = (size_t)2 * 2 * 64 * 64 * sizeof(bf16_t);
  if (a.causal) flash64x2_kernel<true><<<grid, 256, lds, s>>>(a);
  else flash64x2_kernel<false><<<grid, 256, lds, s>>>(a);
}

// flash128x2: flash64x2's structure at D = 128 (Flux joint attention: 24 heads x 128 over 1056-4608 tokens; Llama /
// Mistral prefill) -- the round-5 verdict's ask for the 8-wave ping-pong flash2<128> (40 % MFMA busy).  Four waves of
// two 32-query groups each (256 queries per workgroup, ONE workgroup per CU: ~400 registers per lane).  Per 64-key
// tile every K fragment (16 ds_read_b128) and every V^T fragment (32 transposed reads) is read ONCE and feeds both
// groups' MFMAs; group B's score MFMAs and A's P.V MFMAs sit in the same basic block as the other group's branch-free
// exponentials (one wave per SIMD interleaves its own MFMA and VALU streams).  Per tile and wave: 2 x (2 x 9 + 16) =
// 68 32x32x16 MFMAs (~2.2k matrix cycles) vs ~0.9k cycles of softmax VALU.  K / V tiles (16 KB each) by LDS-DMA into a
// 3-slot ring, two tiles ahead (vmcnt counted: tile t + 2's 8 DMAs per wave stay in flight), source-side XOR
// swizzles as flash2<128> (K: chunk ^ (row & 15); V: chunk ^ ((row & 3) << 2)).
// Measured (round 6, tools/bench_attn128.py): 11-15 % SLOWER than flash2<128> (Flux 1024^2 312 vs 278 us): the
// kernel needs ~400 registers (256 VGPR + 144 AGPR, accumulators shuffled between the files) and one wave per SIMD
// does not hide its own softmax; kept opt-in (SHAI_FLASH128X2=1) with its tests.
__device__ __forceinline__ int f4_kswz(int row, int ch) { return row * 128 + ((ch ^ (row & 15)) << 3); }
__device__ __forceinline__ int f4_vswz(int row, int ch) { return row * 128 + ((ch ^ ((row & 3) << 2)) << 3); }
__device__ __forceinline__ void f4_glds(__amdgpu_buffer_rsrc_t r, bf16_t* lds, uint32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (f3_lds_void*)lds, 16, off, 0, 0, 0);
}

template <bool CAUSAL>
__global__ void __launch_bounds__(256, 1) flash128x2_kernel(const AttnArgs p) {
  constexpr int D = 128, KT = 64, NS = 8, ND = 4, G = 2, NSLOT = 3;
  constexpr int TILE = 2 * KT * D;   // ring slot: K tile then V tile (elements)
  constexpr float kSumThr = 256.f;
  constexpr float kL2e = 1.4426950408889634f;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 31, fh = lane >> 5;
  const int b = blockIdx.z, hq = blockIdx.y;
  const int hk = hq / (p.Hq / p.Hkv);
  const int q_len = p.q_lens ? p.q_lens[b] : p.Sq;
  const int kv_len = p.kv_lens ? p.kv_lens[b] : p.Skv;
  const int c_off = p.q_lens ? kv_len - q_len : p.causal_offset;
  if ((int)blockIdx.x * 256 >= q_len) return;
  const int q0 = blockIdx.x * 256;
  int qi[G];
#pragma unroll
  for (int g = 0; g < G; ++g) qi[g] = q0 + wid * 64 + 32 * g + fr;
  const float sl2 = p.scale * kL2e;

  const bf16_t* kbase = p.k + (long)b * p.k_bs + (long)hk * D;
  const bf16_t* vbase = p.v + (long)b * p.v_bs + (long)hk * D;
  // descriptors sized to the valid keys: rows past kv_len read as zeros (never NaN garbage into P.V)
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(kbase), (short)0, (int)min((long)kv_len * p.k_ts * 2, 0x7fffffffL), 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(vbase), (short)0, (int)min((long)kv_len * p.v_ts * 2, 0x7fffffffL), 0x00020000);
  int kv_end = kv_len;
  if (CAUSAL) kv_end = min(kv_end, q0 + 255 + c_off + 1);
  const int ntiles = kv_end > 0 ? (kv_end + KT - 1) / KT : 0;
  // DMA: wave wid stages K rows 16 wid + 4 j + (lane >> 4) and the same V rows (j < 4), 16 B chunk lane & 15
  const int drow = wid * 16 + (lane >> 4), dch = lane & 15;
  uint32_t koffs[4], voffs[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = drow + 4 * j;
    koffs[j] = (uint32_t)(((long)row * p.k_ts + ((dch ^ (row & 15)) * 8)) * 2);
    voffs[j] = (uint32_t)(((long)row * p.v_ts + ((dch ^ ((row & 3) << 2)) * 8)) * 2);
  }
  auto dma = [&](int slot, int t) {
    bf16_t* ks = smem + slot * TILE;
    bf16_t* vs = ks + KT * D;
    const uint32_t tk = (uint32_t)((long)t * KT * p.k_ts * 2), tv = (uint32_t)((long)t * KT * p.v_ts * 2);
    SHAI_DASSERT(slot >= 0 && slot < NSLOT);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f4_glds(rk, ks + (wid * 16 + 4 * j) * D, koffs[j] + tk);
      f4_glds(rv, vs + (wid * 16 + 4 * j) * D, voffs[j] + tv);
    }
  };
  // tiles 0 and 1 in flight (over-issued past the end: zero fill, never read)
  dma(0, 0);
  dma(1, 1);

  f3bf16x8 qf[G][NS];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const bf16_t* qp = p.q + (p.q_start ? (long)p.q_start[b] * p.q_ts : (long)b * p.q_bs) +
                        (long)min(qi[g], q_len - 1) * p.q_ts + (long)hq * D;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      uint4_ v = *reinterpret_cast<const uint4_*>(qp + 16 * s + 8 * fh);
      if (qi[g] >= q_len) v = uint4_{0u, 0u, 0u, 0u};
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= sl2;
      qf[g][s] = __builtin_bit_cast(f3bf16x8, pack8(f));
    }
  }

  float16_ o[G][ND];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[g][d][r] = 0.f;
  float m_run[G], l_run[G];
  f3bf16x8 b_negm[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m_run[g] = -INFINITY;
    l_run[g] = 0.f;
    b_negm[g] = __builtin_bit_cast(f3bf16x8, uint4_{0u, 0u, 0u, 0u});
  }
  const f3bf16x8 a_one = __builtin_bit_cast(f3bf16x8, uint4_{lane < 32 ? 0x3F80u : 0u, 0u, 0u, 0u});

  const int g16 = lane >> 4, i16 = lane & 15;
  const int tq = i16 >> 2, tp = i16 & 3;
  int koff[NS], voff[ND];
#pragma unroll
  for (int s = 0; s < NS; ++s) koff[s] = f4_kswz(fr, 2 * s + fh);
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    const int col = d * 32 + 16 * (g16 & 1) + 4 * tp;
    voff[d] = f4_vswz(4 * fh + tq, col >> 3) + 4 * ((col >> 2) & 1);
  }

  float16_ sacc[G][2];
  f3bf16x8 pf[G][2][2];
  auto expo = [&](int g, float add, auto addt) {
    constexpr bool ADD = decltype(addt)::value;
    float ls4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          e[j] = __builtin_amdgcn_exp2f(ADD ? sacc[g][kb][8 * s + j] + add : sacc[g][kb][8 * s + j]);
        f3bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          ls4[j & 3] += e[j];
          v[j] = (__bf16)e[j];
        }
        pf[g][kb][s] = v;
      }
    return (ls4[0] + ls4[1]) + (ls4[2] + ls4[3]);
  };
  // slow path of group g (masking, lazy-max rescale) after the branch-free fast path, as flash64x2
  auto check = [&](int g, int key0, float ls_fast) {
    const bool mask = (key0 + KT > kv_len) || (CAUSAL && key0 + KT - 1 > q0 + wid * 64 + 32 * g + c_off);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) asm volatile("" ::"v"(pf[g][kb][s2]));
    asm volatile("" ::"v"(ls_fast));
    const uint64_t slow_lanes = __ballot(m_run[g] == -INFINITY) | __ballot(!(ls_fast <= kSumThr));
    float ls = ls_fast;
    if (mask | (slow_lanes != 0)) {
      if (mask) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = key0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
            const bool bad = key >= kv_len || (CAUSAL && key > qi[g] + c_off);
            sacc[g][kb][r] = bad ? -INFINITY : sacc[g][kb][r];
          }
      }
      float m4[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) m4[r & 3] = fmaxf(m4[r & 3], sacc[g][kb][r]);
      const float mb = m_run[g] == -INFINITY ? 0.f : m_run[g];
      float mloc = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64)) + mb;
      uint32_t u = __float_as_uint(fmaxf(m_run[g], mloc));
      if ((u & 0xffffu) != 0u && u != 0xff800000u) u = (u & 0x80000000u) ? (u & 0xffff0000u) : ((u + 0x10000u) & 0xffff0000u);
      const float m_new = __uint_as_float(u);
      const float m_use = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f(m_run[g] - m_use);
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[g][d][r] *= alpha;
      l_run[g] *= alpha;
      const float shift = mb - m_use;
      m_run[g] = m_new;
      const uint32_t nb = __float_as_uint(-(m_run[g] == -INFINITY ? 0.f : m_run[g])) >> 16;
      b_negm[g] = __builtin_bit_cast(f3bf16x8, uint4_{lane < 32 ? nb : 0u, 0u, 0u, 0u});
      ls = expo(g, shift, std::true_type{});
    }
    l_run[g] += ls;
  };

  for (int t = 0; t < ntiles; ++t) {
    const int cur = t % NSLOT;
    // tile t landed (this wave's 8 DMAs of tile t + 1 stay in flight), every wave past its reads of slot (t + 2) % 3
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    dma((t + 2) % NSLOT, t + 2);
    const bf16_t* ks = smem + cur * TILE;
    const bf16_t* vs = ks + KT * D;
    const int key0 = t * KT;
    // scores of both groups: every K fragment read once
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const float16_ z = {};
#pragma unroll
      for (int g = 0; g < G; ++g) sacc[g][kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_one, b_negm[g], z, 0, 0, 0);
#pragma unroll
      for (int s2 = 0; s2 < NS; ++s2) {
        const f3bf16x8 kf = *reinterpret_cast<const f3bf16x8*>(ks + koff[s2] + kb * 32 * D);
#pragma unroll
        for (int g = 0; g < G; ++g) sacc[g][kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[g][s2], sacc[g][kb], 0, 0, 0);
      }
    }
    const float ls0 = expo(0, 0.f, std::false_type{});
    check(0, key0, ls0);
    // P.V of group A beside group B's exponentials; each V^T fragment read once for both groups
    f3bf16x8 vf[ND][2][2];
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16_t* a0 = vs + voff[d] + kb * 32 * D + s2 * 16 * D;
          const f3s4v t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) f3s4v*)(a0));
          const f3s4v t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) f3s4v*)(a0 + 8 * D));
          vf[d][kb][s2] = __builtin_bit_cast(f3bf16x8, __builtin_shufflevector(t0, t1, 0, 1, 2, 3, 4, 5, 6, 7));
          o[0][d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[d][kb][s2], pf[0][kb][s2], o[0][d], 0, 0, 0);
        }
    const float ls1 = expo(1, 0.f, std::false_type{});
    check(1, key0, ls1);
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          o[1][d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[d][kb][s2], pf[1][kb][s2], o[1][d], 0, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the over-issued tail DMAs land before the workgroup exits

#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float l_tot = l_run[g] + __shfl_xor(l_run[g], 32, 64);
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    if (qi[g] < q_len) {
      bf16_t* op = p.o + (p.q_start ? (long)p.q_start[b] * p.o_ts : (long)b * p.o_bs) + (long)qi[g] * p.o_ts +
                   (long)hq * D;
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          const int dd = d * 32 + 8 * gg + 4 * fh;
          uint2_ w;
          w[0] = pack2(o[g][d][4 * gg] * inv, o[g][d][4 * gg + 1] * inv);
          w[1] = pack2(o[g][d][4 * gg + 2] * inv, o[g][d][4 * gg + 3] * inv);
          *reinterpret_cast<uint2_*>(op + dd) = w;
        }
    }
  }
}

// D = 128, no additive bias / paged K/V, 16-B aligned rows; causal (+ offset), per-batch q / kv lengths, packed
// varlen q / o and GQA as flash2
bool flash128x2_supported(const AttnArgs& a) {
  return a.D == 128 && a.bias == nullptr && a.block_table == nullptr && ((a.k_ts | a.v_ts | a.q_ts) & 7) == 0 &&
         (long)a.Skv * a.k_ts * 2 < 0x7fffffffL && (long)a.Skv * a.v_ts * 2 < 0x7fffffffL;
}

void launch_flash128x2(const AttnArgs& a, hipStream_t s) {
  dim3 grid((a.Sq + 255) / 256, a.Hq, a.B);
  const size_t lds = (size_t)3 * 2 * 64 * 128 * sizeof(bf16_t);   // 96 KB: 3 ring slots of K + V
  if (a.causal) flash128x2_kernel<true><<<grid, 256, lds, s>>>(a);
  else flash128x2_kernel<false><<<grid, 256, lds, s>>>(a);
}

// Same contract as flash64 (attention.hip): D = 64, causal (+ offset), per-batch q / kv lengths, packed varlen
// q / o, GQA; K / V rows addressed through 32-bit buffer offsets.
bool flash64_dma_supported(const AttnArgs& a) {
  return a.D == 64 && a.bias == nullptr && a.block_table == nullptr && ((a.k_ts | a.v_ts | a.q_ts) & 7) == 0 &&
         (long)a.Skv * a.k_ts * 2 < 0x7fffffffL && (long)a.Skv * a.v_ts * 2 < 0x7fffffffL;
}

void launch_flash64_dma(const AttnArgs& a, hipStream_t s) {
  dim3 grid((a.Sq + 127) / 128, a.Hq, a.B);
  const size_t lds = (size_t)2 * 2 * 64 * 64 * sizeof(bf16_t);
  if (a.causal) flash64_dma_kernel<2, true><<<grid, 256, lds, s>>>(a);
  else flash64_dma_kernel<2, false><<<grid, 256, lds, s>>>(a);
}

}  // namespace shai

namespace shai {

// ----------------------------------------------------------------------------------------------------------
// attn512: single-head attention with D = 512 -- the VAE mid-block self-attention (SD2.1 / Flux decoders:
// 512 channels, one head, S = (H/8) x (W/8) latent pixels: 4096 at 512^2, 9216 at 768^2).  Fused flash
// form instead of score GEMM -> softmax -> value GEMM: no S x S scores in HBM (the unfused path wrote up to
// 512 MiB of score chunks per call).
//
// * Workgroup = 8 waves x 16 queries; each wave keeps its Q^T fragments (16 x 512, pre-scaled by
//   scale * log2 e, 64 VGPRs) and O^T (512 x 16 fp32, 128 accumulators) in registers.
// * K / V tiles of 32 keys x 512 (32 KB each) staged by LDS-DMA (one 1-KB row per wave-instruction),
//   2-stage ring (128 KB); 16-B chunks XOR-swizzled on the source address: K by (key & 15) -> the
//   ds_read_b128 A fragments are conflict-free; V by 2 (key & 3) + 8 ((key >> 2) & 1) -> the
//   ds_read_b64_tr_b16 transposed reads (V^T fragments) are conflict-free per 32-lane half.
// * S^T = K Q^T on v_mfma_f32_16x16x32_bf16: lane (query fq, group g) holds keys 4g..4g+3 of both 16-key
//   blocks, which is exactly the B fragment P^T of the PV MFMA under the key order k' = 8g + j ->
//   {4g + j, 16 + 4g + j - 4}: P feeds the PV MFMA from registers, no shuffles; the V^T fragment reads use
//   the same key order.
// * Online softmax in the exp2 domain with a deferred max: O / l are rescaled only when a query's tile max
//   exceeds the running max by more than 2^8 (P <= 256 in bf16 otherwise).
constexpr int A5_D = 512, A5_KT = 32, A5_WAVES = 8;
constexpr int A5_STAGE = 2 * A5_KT * A5_D;  // bf16 elements: K tile then V tile

__device__ __forceinline__ int a5_vswz(int r) { return 2 * (r & 3) + 8 * ((r >> 2) & 1); }

__global__ void __launch_bounds__(512, 1) attn512_kernel(const AttnArgs p) {
  constexpr float kThr = 8.f, kL2e = 1.4426950408889634f;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fq = lane & 15, g = lane >> 4;
  const int b = blockIdx.y;
  const int S = p.Skv;
  const int qi = blockIdx.x * 128 + wid * 16 + fq;
  const int nt = (S + A5_KT - 1) / A5_KT;

  const bf16_t* kb_ = p.k + (long)b * p.k_bs;
  const bf16_t* vb_ = p.v + (long)b * p.v_bs;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(kb_), (short)0,
                                                                      0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(vb_), (short)0,
                                                                      0x7fffffff, 0x00020000);
  // DMA: wave w moves K rows 4w .. 4w+3 and V rows 4w .. 4w+3 of each tile (one 1-KB row per instruction)
  auto dma = [&](int stage, int t) {
    bf16_t* ks = smem + stage * A5_STAGE;
    bf16_t* vs = ks + A5_KT * A5_D;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wid * 4 + i, key = t * A5_KT + r;
      const uint32_t oob = key < S ? 0u : 0x80000000u;
      const uint32_t ko = (uint32_t)(((long)key * p.k_ts + ((lane ^ (r & 15)) << 3)) * 2) | oob;
      const uint32_t vo = (uint32_t)(((long)key * p.v_ts + ((lane ^ a5_vswz(r)) << 3)) * 2) | oob;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (f3_lds_void*)(ks + r * A5_D), 16, ko, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (f3_lds_void*)(vs + r * A5_D), 16, vo, 0, 0, 0);
    }
  };
  if (nt > 0) dma(0, 0);

  // Q^T fragments: lane (fq, g) holds q[qi][32 ds + 8 g .. + 8] * scale * log2 e
  f3bf16x8 qf[16];
  {
    const float sl2 = p.scale * kL2e;
    const bf16_t* qp = p.q + (long)b * p.q_bs + (long)min(qi, p.Sq - 1) * p.q_ts + 8 * g;
#pragma unroll
    for (int ds = 0; ds < 16; ++ds) {
      uint4_ v = *reinterpret_cast<const uint4_*>(qp + 32 * ds);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= sl2;
      qf[ds] = __builtin_bit_cast(f3bf16x8, pack8(f));
    }
  }
  // per-lane LDS byte offsets: K fragment (row fq, chunk (4 ds + g) ^ fq; the XOR reaches chunk bits 0-3, i.e.
  // ds & 3) = koff[ds & 3] + 256 (ds >> 2); V^T fragment of d-block db (rows 4g + q (+16), chunk
  // (2 db + (p >> 1)) ^ vswz; vswz reaches chunk bits 1-3, i.e. db & 7) = voff[db & 7] + 256 (db >> 3)
  const int fh = fq >> 2, tq = fq >> 2, tp = lane & 3;
  int koff[4];
#pragma unroll
  for (int bb = 0; bb < 4; ++bb) koff[bb] = fq * A5_D * 2 + ((((bb ^ fh) << 2) | ((g ^ fq) & 3)) << 4);
  // V: chunk position (2 db + (p >> 1)) ^ vswz = 2 (db & 7) ^ vx + 16 (db >> 3), vx = (p >> 1) ^ vswz (one XOR
  // per read instead of 8 more offset registers)
  const int vrow = (4 * g + tq) * A5_D * 2 + (tp & 1) * 8;
  const int vx = (tp >> 1) ^ a5_vswz(4 * g + tq);

  float4_ o[32];
  float m_run = -INFINITY, l_lane = 0.f;
  bool first = true;
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < nt) dma(cur ^ 1, t + 1);
    const char* ks = reinterpret_cast<const char*>(smem + cur * A5_STAGE);
    const char* vs = ks + A5_KT * A5_D * 2;
    int vxl = vx, vrl = vrow;   // opaque per tile: the 32 V^T read addresses are rebuilt, not hoisted into registers
    asm volatile("" : "+v"(vxl), "+v"(vrl));
    float4_ s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const float4_ z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < 16; ++ds) {
        const f3bf16x8 kf = *reinterpret_cast<const f3bf16x8*>(ks + koff[ds & 3] + 256 * (ds >> 2) + kb * 16 * A5_D * 2);
        s[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ds], ds == 0 ? z : s[kb], 0, 0, 0);
      }
    }
    const int key0 = t * A5_KT;
    if (key0 + A5_KT > S) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[kb][r] = key0 + kb * 16 + 4 * g + r < S ? s[kb][r] : -INFINITY;
    }
    float mt = fmaxf(fmaxf(fmaxf(s[0][0], s[0][1]), fmaxf(s[0][2], s[0][3])),
                     fmaxf(fmaxf(s[1][0], s[1][1]), fmaxf(s[1][2], s[1][3])));
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    if (__any(mt > m_run + kThr)) {  // deferred max: rescale only on a large jump (or the first tile)
      const float m_new = fmaxf(m_run, mt);
      const float alpha = m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_run - m_new);
      if (!first) {
#pragma unroll
        for (int db = 0; db < 32; ++db) o[db] *= alpha;
      }
      l_lane *= alpha;
      m_run = m_new;
    }
    const float mu = m_run == -INFINITY ? 0.f : m_run;
    f3bf16x8 pf;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = __builtin_amdgcn_exp2f(s[kb][r] - mu);
        l_lane += e;
        pf[4 * kb + r] = (__bf16)e;
      }
#pragma unroll
    for (int db = 0; db < 32; ++db) {
      const char* a0 = vs + vrl + (((2 * (db & 7)) ^ vxl) << 4) + 256 * (db >> 3);
      const f3s4v t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) f3s4v*)(a0));
      const f3s4v t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) f3s4v*)(a0 + 16 * A5_D * 2));
      short8 vv;
      vv[0] = t0[0]; vv[1] = t0[1]; vv[2] = t0[2]; vv[3] = t0[3];
      vv[4] = t1[0]; vv[5] = t1[1]; vv[6] = t1[2]; vv[7] = t1[3];
      const float4_ z = {0.f, 0.f, 0.f, 0.f};
      o[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(f3bf16x8, vv), pf, first ? z : o[db], 0, 0, 0);
    }
    first = false;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this stage's reads done before it is restaged
  }

  float l = l_lane + __shfl_xor(l_lane, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (qi < p.Sq && nt > 0) {
    bf16_t* op = p.o + (long)b * p.o_bs + (long)qi * p.o_ts + 4 * g;
#pragma unroll
    for (int db = 0; db < 32; ++db) {
      uint2_ w;
      w[0] = pack2(o[db][0] * inv, o[db][1] * inv);
      w[1] = pack2(o[db][2] * inv, o[db][3] * inv);
      *reinterpret_cast<uint2_*>(op + 16 * db) = w;
    }
  }
}

bool attn512_supported(const AttnArgs& a) {
  return a.D == 512 && a.Hq == 1 && a.Hkv == 1 && a.Sq == a.Skv && a.bias == nullptr && a.block_table == nullptr &&
         !a.causal && a.kv_lens == nullptr && a.q_lens == nullptr && a.q_start == nullptr &&
         ((a.k_ts | a.v_ts | a.q_ts | a.o_ts) & 7) == 0 && (long)a.Skv * a.k_ts * 2 < 0x7fffffffL &&
         (long)a.Skv * a.v_ts * 2 < 0x7fffffffL;
}

void launch_attn512(const AttnArgs& a, hipStream_t s) {
  dim3 grid((a.Sq + 127) / 128, a.B);
  attn512_kernel<<<grid, 512, (size_t)2 * A5_STAGE * sizeof(bf16_t), s>>>(a);
}

}  // namespace shai
