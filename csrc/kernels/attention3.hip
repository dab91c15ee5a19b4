// flash64 with LDS-DMA K/V staging (lab variant, `launch_flash64_dma`): the register-staged K/V pipeline of
// flash64 (attention.hip) holds 16 VGPRs of next-tile K/V plus the ds_write pass; staging the tiles with
// `buffer_load ... lds` (source-side swizzle, lane-linear LDS image) frees them, and the softmax computes P in
// chunks of 8 exponentials instead of a 32-float buffer, so the kernel can aim at 4 waves per SIMD (128 VGPRs)
// instead of 3 (168): more co-resident waves to overlap one wave's MFMAs with another's softmax, which is what
// bounds D = 64 attention (VALU issue + latency, profiles/pmc_round3.md: 37 % MFMA busy).
#include "common.h"
#include "launchers.h"

#include <type_traits>

namespace shai {

typedef __bf16 f3bf16x8 __attribute__((ext_vector_type(8)));
typedef short f3s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void f3_lds_void;

__device__ __forceinline__ int f3_kswz(int row, int ch) { return row * 64 + ((ch ^ ((row >> 1) & 7)) << 3); }
__device__ __forceinline__ int f3_vswz(int row, int ch) { return row * 64 + ((ch ^ (((row >> 1) & 1) << 2)) << 3); }

template <int OCC>
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
  const int q_len = p.Sq, kv_len = p.Skv;
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
  const int ntiles = (kv_len + KT - 1) / KT;
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
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (f3_lds_void*)(ks + (wid * 16) * D), 16, (r0 + kch0 * 16) | ok0, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (f3_lds_void*)(ks + (wid * 16 + 8) * D), 16, (r1 + kch1 * 16) | ok1, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (f3_lds_void*)(vs + (wid * 16) * D), 16, (v0 + vch0 * 16) | ok0, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (f3_lds_void*)(vs + (wid * 16 + 8) * D), 16, (v1 + vch1 * 16) | ok1, 0, 0, 0);
  };
  if (ntiles > 0) dma(0, 0);

  f3bf16x8 qf[NS];
  {
    const bf16_t* qp = p.q + (long)b * p.q_bs + (long)min(qi, q_len - 1) * p.q_ts + (long)hq * D;
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
    if (key0 + KT > kv_len) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = key0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          sacc[kb][r] = key >= kv_len ? -INFINITY : sacc[kb][r];
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
    bf16_t* op = p.o + (long)b * p.o_bs + (long)qi * p.o_ts + (long)hq * D;
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

bool flash64_dma_supported(const AttnArgs& a) {
  return a.D == 64 && a.bias == nullptr && a.block_table == nullptr && !a.causal && a.kv_lens == nullptr &&
         a.q_lens == nullptr && a.q_start == nullptr && ((a.k_ts | a.v_ts | a.q_ts) & 7) == 0 &&
         (long)a.Skv * a.k_ts * 2 < 0x7fffffffL && (long)a.Skv * a.v_ts * 2 < 0x7fffffffL;
}

void launch_flash64_dma(const AttnArgs& a, int occ, hipStream_t s) {
  dim3 grid((a.Sq + 127) / 128, a.Hq, a.B);
  const size_t lds = (size_t)2 * 2 * 64 * 64 * sizeof(bf16_t);
  if (occ >= 4) flash64_dma_kernel<4><<<grid, 256, lds, s>>>(a);
  else flash64_dma_kernel<2><<<grid, 256, lds, s>>>(a);
}

}  // namespace shai
