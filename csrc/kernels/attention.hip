// Attention kernels for gfx950.
//
// flash_attn_fwd: fused QK^T -> online softmax -> PV on MFMA (no S x S matrix
//   in HBM; replaces the reference's attention slicing / NEURON_FUSE_SOFTMAX
//   paths, app/run-sd.py:135, app/compile-sd2.py:2).  One workgroup = 4 waves
//   = 128 query rows; each wave owns 32 queries.  Scores are computed swapped
//   (S^T = K Q^T, v_mfma_f32_32x32x16_bf16) so every lane holds one query's
//   scores: the row max / row sum are in-lane plus one cross-half shuffle.
//   P stays in registers and feeds O^T = V^T P^T directly as the B operand
//   (accumulator-as-operand); V^T fragments come from ds_read_b64_tr_b16
//   transposed LDS reads of the row-major V tile.  K/V tiles (64 keys) are
//   register-staged one tile ahead and double-buffered in XOR-swizzled LDS.
//   Supports D in {64,128}, GQA, causal (with offset for chunked prefill),
//   per-batch q/kv lengths (padding masks), additive bias (T5 relative
//   position bias) and a paged K/V source (64-token blocks).
//
// decode_attn: one query token per sequence against the paged KV cache,
//   split-K over 64-token blocks (memory-bound; VALU dot products, K/V
//   staged through LDS), followed by a split combine.
#include "common.h"
#include "launchers.h"

#include <algorithm>

#include <cstdlib>
#include <type_traits>

namespace shai {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kRescaleThr = 8.f;   // flash_fwd deferred-max threshold (log2 units)

template <int D>
__device__ __forceinline__ int k_swz(int row, int ch) {
  if constexpr (D == 128) return row * 128 + ((ch ^ (row & 15)) << 3);
  else return row * 64 + ((ch ^ ((row >> 1) & 7)) << 3);
}
template <int D>
__device__ __forceinline__ int v_swz(int row, int ch) {
  if constexpr (D == 128) return row * 128 + ((ch ^ ((row & 3) << 2)) << 3);
  else return row * 64 + ((ch ^ (((row >> 1) & 1) << 2)) << 3);
}

template <int D>
__global__ void __launch_bounds__(256, 2) flash_fwd_kernel(const AttnArgs p) {
  constexpr int KT = 64;                 // keys per tile
  constexpr int CPR = D / 8;             // 16-byte chunks per row
  constexpr int NST = KT * CPR / 256;    // chunks per thread per operand
  constexpr int NS = D / 16;             // k-steps for QK^T
  constexpr int ND = D / 32;             // 32-wide d blocks of O
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  bf16_t* sK = smem;                     // [2][64*D]
  bf16_t* sV = smem + 2 * KT * D;        // [2][64*D]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 31, fh = lane >> 5;
  const int b = blockIdx.z, hq = blockIdx.y;
  const int hk = hq / (p.Hq / p.Hkv);
  const int q_len = p.q_lens ? p.q_lens[b] : p.Sq;
  const int kv_len = p.kv_lens ? p.kv_lens[b] : p.Skv;
  const int c_off = p.q_lens ? kv_len - q_len : p.causal_offset;
  if ((int)blockIdx.x * 128 >= q_len) return;
  const int q0 = blockIdx.x * 128;
  const int qi = q0 + wid * 32 + fr;  // this lane's query

  // ---- Q fragments (B operand of S^T = K Q^T): Q[qi][16 s + 8 fh .. +7]
  bf16x8 qf[NS];
  {
    const bf16_t* qp = p.q + (p.q_start ? (long)p.q_start[b] * p.q_ts : (long)b * p.q_bs) +
                        (long)min(qi, q_len - 1) * p.q_ts + (long)hq * D;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      uint4_ v = *reinterpret_cast<const uint4_*>(qp + 16 * s + 8 * fh);
      if (qi >= q_len) v = uint4_{0u, 0u, 0u, 0u};
      qf[s] = __builtin_bit_cast(bf16x8, v);
    }
  }

  // ---- number of key tiles this block needs
  int kv_end = kv_len;
  if (p.causal) kv_end = min(kv_end, q0 + 127 + c_off + 1);
  const int ntiles = kv_end > 0 ? (kv_end + KT - 1) / KT : 0;

  const bf16_t* kbase = p.k + (long)b * p.k_bs + (long)hk * D;
  const bf16_t* vbase = p.v + (long)b * p.v_bs + (long)hk * D;

  uint4_ rk[NST], rv[NST];
  auto load_tile = [&](int t) {
    const int key0 = t * KT;
    const bf16_t* kb = kbase;
    const bf16_t* vb = vbase;
    long ts_k = p.k_ts, ts_v = p.v_ts;
    int kbase_row = key0;
    if (p.block_table) {
      const int phys = p.block_table[(long)b * p.max_blocks + t];
      kb = p.k + (long)phys * p.kc_bs + (long)hk * p.kc_hs;
      vb = p.v + (long)phys * p.kc_bs + (long)hk * p.kc_hs;
      ts_k = ts_v = D;
      kbase_row = 0;
    }
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int id = tid + 256 * i;
      const int row = id / CPR, ch = id % CPR;
      const bool ok = key0 + row < kv_len;
      rk[i] = ok ? *reinterpret_cast<const uint4_*>(kb + (long)(kbase_row + row) * ts_k + ch * 8) : uint4_{0u, 0u, 0u, 0u};
      rv[i] = ok ? *reinterpret_cast<const uint4_*>(vb + (long)(kbase_row + row) * ts_v + ch * 8) : uint4_{0u, 0u, 0u, 0u};
    }
  };
  auto store_tile = [&](int stage) {
    bf16_t* ks = sK + stage * KT * D;
    bf16_t* vs = sV + stage * KT * D;
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int id = tid + 256 * i;
      const int row = id / CPR, ch = id % CPR;
      *reinterpret_cast<uint4_*>(ks + k_swz<D>(row, ch)) = rk[i];
      *reinterpret_cast<uint4_*>(vs + v_swz<D>(row, ch)) = rv[i];
    }
  };

  float16_ o[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  const float sl2 = p.scale * kLog2e;
  const bf16_t* bias_row = p.bias ? p.bias + ((long)hq * p.Sq + min(qi, q_len - 1)) * p.Skv : nullptr;

  if (ntiles > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();

  // lane roles for the transposed V reads
  const int g16 = lane >> 4, i16 = lane & 15;
  const int tq = i16 >> 2, tp = i16 & 3;

  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) load_tile(t + 1);
    const bf16_t* ks = sK + cur * KT * D;
    const bf16_t* vs = sV + cur * KT * D;

    // ---- S^T = K Q^T for two 32-key blocks
    float16_ sacc[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[kb][r] = 0.f;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(ks + k_swz<D>(kb * 32 + fr, 2 * s + fh));
        sacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc[kb], 0, 0, 0);
      }
    }
    // ---- mask (+ bias), row max on raw scores, exp2 with the scale folded into one FMA
    const int key0 = t * KT;
    const bool need_mask = (key0 + KT > kv_len) || (p.causal && key0 + KT - 1 > q0 + c_off);
    float mloc = -INFINITY;
    if (bias_row) {  // T5 relative-position bias: additive in the natural-log domain
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = key0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          sacc[kb][r] += (key < p.Skv ? bf2f(bias_row[key]) : 0.f) / p.scale;
        }
    }
    if (need_mask) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = key0 + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          const bool bad = key >= kv_len || (p.causal && key > qi + c_off);
          sacc[kb][r] = bad ? -INFINITY : sacc[kb][r];
        }
    }
    {  // 4 independent max chains (a single chain is 32 dependent v_max on the critical path)
      float m4[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) m4[r & 3] = fmaxf(m4[r & 3], sacc[kb][r]);
      mloc = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64)) * sl2;   // scale > 0: max commutes with scaling
    // Deferred max: keep the running max (and skip the O rescale) unless some row's max grew by more
    // than kRescaleThr (log2 units) -- P is then bounded by 2^kRescaleThr instead of 1, which the bf16 P /
    // fp32 O, l accumulators absorb; the decision precedes this tile's exponentials, so everything still at
    // the old max is rescaled exactly once.
    const float m_cand = fmaxf(m_run, mloc);
    const bool grew = __any(m_cand > m_run + kRescaleThr);
    const float m_keep = grew ? m_cand : m_run;
    const float m_use = m_keep == -INFINITY ? 0.f : m_keep;
    const float alpha = grew ? __builtin_amdgcn_exp2f(m_run - m_use) : 1.f;
    m_run = m_keep;
    float ls4[4] = {0.f, 0.f, 0.f, 0.f};  // independent partial row sums (ILP)
    bf16x8 pf[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(fmaf(sacc[kb][r], sl2, -m_use));
        sacc[kb][r] = e;
        ls4[r & 3] += e;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (__bf16)sacc[kb][8 * s + j];
        pf[kb][s] = v;
      }
    }
    const float lsum = (ls4[0] + ls4[1]) + (ls4[2] + ls4[3]);
    l_run = l_run * alpha + lsum;
    if (grew) {
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[d][r] *= alpha;
    }

    // ---- O^T += V^T P^T
#pragma unroll
    for (int d = 0; d < ND; ++d) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int r0 = kb * 32 + 16 * s + 4 * fh + tq;
          const int col = d * 32 + 16 * (g16 & 1) + 4 * tp;
          const int ch = col >> 3, half = (col >> 2) & 1;
          const bf16_t* a0 = vs + v_swz<D>(r0, ch) + 4 * half;
          const bf16_t* a1 = vs + v_swz<D>(r0 + 8, ch) + 4 * half;
          const s4v t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(a0));
          const s4v t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(a1));
          short8 vv;
          vv[0] = t0[0]; vv[1] = t0[1]; vv[2] = t0[2]; vv[3] = t0[3];
          vv[4] = t1[0]; vv[5] = t1[1]; vv[6] = t1[2]; vv[7] = t1[3];
          o[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, vv), pf[kb][s], o[d], 0, 0, 0);
        }
      }
    }
    if (t + 1 < ntiles) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qi < q_len) {
    bf16_t* op = p.o + (p.q_start ? (long)p.q_start[b] * p.o_ts : (long)b * p.o_bs) + (long)qi * p.o_ts +
                 (long)hq * D;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
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
}

// ----------------------------------------------------------------------------
// flash64: the v1 structure above (4 waves x 32 queries, register-staged K/V, double-buffered swizzled
// LDS, several workgroups per CU so that one wave's MFMAs overlap another's softmax) specialised for
// D = 64 without bias / paged K/V -- every SD2.1 attention.  At D = 64 the loop is bound by VALU issue
// (the softmax costs about what the 16 MFMAs of a 64-key tile do), so the VALU per tile is cut from
// ~125 to ~70 instructions:
//  * Q is pre-multiplied by scale * log2(e) (one bf16 rounding of the scaled Q, |rel| <= 2^-9 per element):
//    the scores arrive in the exp2 domain.
//  * -m enters each 32-key score chain as one extra v_mfma (A = a ones column, B = -m; the running max is
//    kept on the bf16 grid so it is exact as a bf16 operand): the accumulators start at the inline constant
//    0 and P = exp2(acc) is one v_exp per score, no FMA / no accumulator initialisation moves.
//  * Max-free fast path (as flash2): the running max stays unchanged while every lane's partial row sum of
//    the tile is <= 2^8 (P then stays bounded by 2^8: bf16 P, fp32 O / l absorb it); otherwise, or before a
//    row has a max, the tile takes the exact path (tile max, O / l rescale, recompute P).
//  * Fragment reads at immediate offsets from six per-stage base addresses (the XOR swizzle depends on
//    the lane only).
template <bool CAUSAL>
__global__ void __launch_bounds__(256, 2) flash64_kernel(const AttnArgs p) {
  constexpr int D = 64, KT = 64, CPR = 8, NST = KT * CPR / 256, NS = 4, ND = 2;
  constexpr float kSumThr = 256.f;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  bf16_t* sK = smem;
  bf16_t* sV = smem + 2 * KT * D;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 31, fh = lane >> 5;
  const int b = blockIdx.z, hq = blockIdx.y;
  const int hk = hq / (p.Hq / p.Hkv);
  const int q_len = p.q_lens ? p.q_lens[b] : p.Sq;
  const int kv_len = p.kv_lens ? p.kv_lens[b] : p.Skv;
  const int c_off = p.q_lens ? kv_len - q_len : p.causal_offset;
  if ((int)blockIdx.x * 128 >= q_len) return;
  const int q0 = blockIdx.x * 128;
  const int qi = q0 + wid * 32 + fr;
  const float sl2 = p.scale * kLog2e;

  bf16x8 qf[NS];
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
      qf[s] = __builtin_bit_cast(bf16x8, pack8(f));
    }
  }

  int kv_end = kv_len;
  if (CAUSAL) kv_end = min(kv_end, q0 + 127 + c_off + 1);
  const int ntiles = kv_end > 0 ? (kv_end + KT - 1) / KT : 0;
  const bf16_t* kbase = p.k + (long)b * p.k_bs + (long)hk * D;
  const bf16_t* vbase = p.v + (long)b * p.v_bs + (long)hk * D;

  uint4_ rk[NST], rv[NST];
  auto load_tile = [&](int t) {
    const int key0 = t * KT;
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int id = tid + 256 * i;
      const int row = id / CPR, ch = id % CPR;
      const bool ok = key0 + row < kv_len;
      rk[i] = ok ? *reinterpret_cast<const uint4_*>(kbase + (long)(key0 + row) * p.k_ts + ch * 8) : uint4_{0u, 0u, 0u, 0u};
      rv[i] = ok ? *reinterpret_cast<const uint4_*>(vbase + (long)(key0 + row) * p.v_ts + ch * 8) : uint4_{0u, 0u, 0u, 0u};
    }
  };
  auto store_tile = [&](int stage) {
    bf16_t* ks = sK + stage * KT * D;
    bf16_t* vs = sV + stage * KT * D;
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int id = tid + 256 * i;
      const int row = id / CPR, ch = id % CPR;
      *reinterpret_cast<uint4_*>(ks + k_swz<D>(row, ch)) = rk[i];
      *reinterpret_cast<uint4_*>(vs + v_swz<D>(row, ch)) = rv[i];
    }
  };

  float16_ o[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  auto m_base = [&]() { return m_run == -INFINITY ? 0.f : m_run; };
  // -m MFMA operands: A[key][k] = (k == 0), B[k][query] = (k == 0) * -m_base (lanes 0-31 hold k 0..7)
  const bf16x8 a_one = __builtin_bit_cast(bf16x8, uint4_{lane < 32 ? 0x3F80u : 0u, 0u, 0u, 0u});
  bf16x8 b_negm = __builtin_bit_cast(bf16x8, uint4_{0u, 0u, 0u, 0u});

  const int g16 = lane >> 4, i16 = lane & 15;
  const int tq = i16 >> 2, tp = i16 & 3;
  int koff[NS], voff[ND];  // element offsets inside a stage (key block 0 / first transposed-read row)
#pragma unroll
  for (int s = 0; s < NS; ++s) koff[s] = k_swz<D>(fr, 2 * s + fh);
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    const int col = d * 32 + 16 * (g16 & 1) + 4 * tp;
    voff[d] = v_swz<D>(4 * fh + tq, col >> 3) + 4 * ((col >> 2) & 1);
  }

  if (ntiles > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();

  float16_ sacc[2];
  bf16x8 pf[2][2];
  // P from the accumulators (+ add when ADD); returns this lane's partial row sum.  All 32 exponentials
  // first: consuming each v_exp result right away pads it with an s_nop (transcendental hazard).
  auto expo = [&](float add, auto addt) {
    constexpr bool ADD = decltype(addt)::value;
    float e[2][16];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) e[kb][r] = __builtin_amdgcn_exp2f(ADD ? sacc[kb][r] + add : sacc[kb][r]);
    __builtin_amdgcn_sched_barrier(0);
    float ls4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          ls4[j & 3] += e[kb][8 * s + j];
          v[j] = (__bf16)e[kb][8 * s + j];
        }
        pf[kb][s] = v;
      }
    return (ls4[0] + ls4[1]) + (ls4[2] + ls4[3]);
  };

  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) load_tile(t + 1);
    const bf16_t* ks = sK + cur * KT * D;
    const bf16_t* vs = sV + cur * KT * D;

    // ---- S^T - m = K Q^T - m for two 32-key blocks
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const float16_ z = {};
      sacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_one, b_negm, z, 0, 0, 0);
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(ks + koff[s] + kb * 2048);
        sacc[kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc[kb], 0, 0, 0);
      }
    }
    const int key0 = t * KT;
    const bool need_mask = (key0 + KT > kv_len) || (CAUSAL && key0 + KT - 1 > q0 + c_off);
    if (need_mask) {
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
    if (slow) {  // exact path: tile max, rescale O and l, recompute P
      float m4[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) m4[r & 3] = fmaxf(m4[r & 3], sacc[kb][r]);
      float mloc = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64)) + m_base();  // accumulators hold s - m_base
      const float m_new = bf16_up(fmaxf(m_run, mloc));
      const float m_use = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);  // 0 when m_run = -inf
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[d][r] *= alpha;
      l_run *= alpha;
      const float shift = m_base() - m_use;
      m_run = m_new;
      const uint32_t nb = __float_as_uint(-m_base()) >> 16;  // bf16-exact
      b_negm = __builtin_bit_cast(bf16x8, uint4_{lane < 32 ? nb : 0u, 0u, 0u, 0u});
      ls = expo(shift, std::true_type{});
    }
    l_run += ls;

    // ---- O^T += V^T P^T
#pragma unroll
    for (int d = 0; d < ND; ++d) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16_t* a0 = vs + voff[d] + kb * 2048 + s * 1024;
          const s4v t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(a0));
          const s4v t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(a0 + 512));
          short8 vv;
          vv[0] = t0[0]; vv[1] = t0[1]; vv[2] = t0[2]; vv[3] = t0[3];
          vv[4] = t1[0]; vv[5] = t1[1]; vv[6] = t1[2]; vv[7] = t1[3];
          o[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, vv), pf[kb][s], o[d], 0, 0, 0);
        }
      }
    }
    if (t + 1 < ntiles) store_tile(cur ^ 1);
    __syncthreads();
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qi < q_len) {
    bf16_t* op = p.o + (p.q_start ? (long)p.q_start[b] * p.o_ts : (long)b * p.o_bs) + (long)qi * p.o_ts +
                 (long)hq * D;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
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
}

bool flash64_supported(const AttnArgs& a) {
  static const bool on = [] {
    const char* e = getenv("SHAI_FLASH64");
    return e == nullptr || atoi(e) != 0;
  }();
  return on && a.D == 64 && a.bias == nullptr && a.block_table == nullptr && ((a.k_ts | a.v_ts | a.q_ts) & 7) == 0;
}

void launch_flash64(const AttnArgs& a, hipStream_t s) {
  static const bool dma = [] {  // SHAI_FLASH64_DMA=0: the register-staged kernel below (A/B)
    const char* e = getenv("SHAI_FLASH64_DMA");
    return e == nullptr || atoi(e) != 0;
  }();
  if (dma && flash64_dma_supported(a)) {
    // two 32-query groups per wave when the 256-query grid still fills the chip several times over
    // (short key ranges -- SD2.1 cross-attention over 77 text tokens -- stay on the 128-query kernel: 123 vs 142 us)
    if ((long)((a.Sq + 255) / 256) * a.Hq * a.B >= 1024 && a.Skv >= 512) launch_flash64_x2(a, s);
    else launch_flash64_dma(a, s);
    return;
  }
  dim3 grid((a.Sq + 127) / 128, a.Hq, a.B);
  const size_t lds = (size_t)4 * 64 * 64 * sizeof(bf16_t);
  if (a.causal) flash64_kernel<true><<<grid, 256, lds, s>>>(a);
  else flash64_kernel<false><<<grid, 256, lds, s>>>(a);
}

// D = 128 routing: 0 = flash2 (default), 1 = flash128x2 (SHAI_FLASH128X2=1, or set_flash128x2 at run time for A/B).
// flash2 stays the default: the two-group kernel measured 11-15 % slower at the Flux / prefill shapes
// (profiles/flash128x2_ab_round6.json: Flux 1024^2 312 vs 278 us) -- at ~400 registers per lane one wave per SIMD
// cannot hide its own softmax behind its MFMAs the way the 8-wave ping-pong's partner wave does.
static int g_f128x2 = -1;
int flash128x2_mode() {
  if (g_f128x2 < 0) {
    const char* e = getenv("SHAI_FLASH128X2");
    g_f128x2 = (e != nullptr && atoi(e) != 0) ? 1 : 0;
  }
  return g_f128x2;
}
int set_flash128x2(int mode) {
  const int prev = flash128x2_mode();
  if (mode >= 0) g_f128x2 = mode;
  return prev;
}

void launch_flash_attn(const AttnArgs& a, hipStream_t s) {
  static const bool v1_only = getenv("SHAI_FLASH_V1") != nullptr;  // A/B and tests: pin the v1 kernel
  if (!v1_only && flash64_supported(a)) {  // D = 64 (every SD2.1 / ViT / BERT attention)
    launch_flash64(a, s);
    return;
  }
  if (!v1_only && flash128x2_mode() && flash128x2_supported(a) && a.Sq >= 512 && a.Skv >= 512) {
    launch_flash128x2(a, s);
    return;
  }
  if (!v1_only && flash2_supported(a)) {  // 8-wave ping-pong kernel (attention2.hip)
    launch_flash2(a, s);
    return;
  }
  dim3 grid((a.Sq + 127) / 128, a.Hq, a.B);
  const size_t lds = (size_t)4 * 64 * a.D * sizeof(bf16_t);
  if (a.D == 128) flash_fwd_kernel<128><<<grid, 256, lds, s>>>(a);
  else flash_fwd_kernel<64><<<grid, 256, lds, s>>>(a);
}

// ----------------------------------------------------------------------------
// Paged decode attention (one query token per sequence).
// grid (B, Hkv, splits); block = G waves (G = Hq/Hkv <= 8), wave w = head hk*G+w.
// ----------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void da_lds_void;
typedef __bf16 bf16x2d __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8d __attribute__((ext_vector_type(8)));
#define DA_PAIR(v, i) __builtin_shufflevector(v, v, 2 * (i), 2 * (i) + 1)

// Decode attention, one workgroup per (sequence, KV head, split): G = Hq/Hkv waves, one query head
// each.  The 64-token K/V blocks stream global -> LDS by LDS-DMA (buffer_load ... lds) into a
// two-slot ring: block i+1's DMA is in flight while block i is consumed (counted vmcnt of NI
// instructions per wave per block + one barrier), so HBM latency hides behind the dot products.
// Per-block buffer descriptors (the cache can exceed 4 GiB) range-check the tail rows past the
// context: zero-filled, since P = 0 times a never-written NaN pattern would poison P.V.
// Split count of one sequence of nblk 64-token blocks when the launch has num_splits: at least kDaMinSplitBlocks
// blocks per split, so that a batch whose factor was raised for one long context (up to 64 splits at 128k) does
// not give every short sequence 64 mostly-empty workgroups and a 64-way combine.
constexpr int kDaMinSplitBlocks = 4;
__device__ __forceinline__ int da_splits(int nblk, int num_splits) {
  return max(1, min(num_splits, (nblk + kDaMinSplitBlocks - 1) / kDaMinSplitBlocks));
}

template <int D, int NI>
__device__ __forceinline__ void decode_attn_item(const DecodeAttnArgs& p, char* dsm, const int b, const int hk,
                                                 const int split) {
  constexpr int CPR = D / 8;
  constexpr int RPI = 1024 / (D * 2);           // K/V rows per 1-KB wave DMA instruction
  constexpr int SLOT = 2 * 64 * D;              // bf16 elements per ring slot (K then V)
  bf16_t* ring = reinterpret_cast<bf16_t*>(dsm);              // [2][K 64xD swizzled | V 64xD linear]
  float* sQ = reinterpret_cast<float*>(ring + 2 * SLOT);      // [G][D]
  float* sP = sQ + 8 * D;                                     // [G][64]
  const int G = p.Hq / p.Hkv;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hq = hk * G + w;
  const bool fused = p.knew != nullptr;
  const int ctx = p.ctx_lens[b] - (fused ? 1 : 0);  // tokens read from the cache
  const int nblk = (ctx + 63) / 64;
  // this sequence's own split count (da_splits): a short sequence in a batch whose split factor was raised for a
  // long one uses one split -- its other workgroups leave here, before any load
  const int nsp = da_splits(nblk, p.num_splits);
  if (split >= nsp) return;
  const int per = (nblk + nsp - 1) / nsp;
  const int blk0 = split * per, blk1 = min(nblk, blk0 + per);

  // wave w issues instructions j = w + G*t (t < NI) of the block's 2 * 64 * D * 2 / 1024 = NI * G
  // physical block ids of this split, 64 per lane-distributed chunk (read ahead, so the ring's
  // DMA issue never waits on a block-table load queued behind the previous block's DMA)
  const int* bt = p.block_table + (long)b * p.max_blocks;
  int chunk0 = blk0;
  int my_phys = (blk0 + lane < blk1) ? bt[blk0 + lane] : 0;
  auto phys_of = [&](int bi) {
    if (bi - chunk0 >= 64) {
      chunk0 += 64;
      my_phys = (chunk0 + lane < blk1) ? bt[chunk0 + lane] : 0;
    }
    return __builtin_amdgcn_readfirstlane(__shfl(my_phys, bi - chunk0, 64));
  };
  auto stage = [&](int slot, int bi) {
    const int phys = phys_of(bi);
    const long base = ((long)phys * p.Hkv + hk) * 64 * D;
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.k_cache + base),
                                                                        (short)0, 64 * D * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(p.v_cache + base),
                                                                        (short)0, 64 * D * 2, 0x00020000);
    bf16_t* dst = ring + slot * SLOT;
#pragma unroll
    for (int t = 0; t < NI; ++t) {
      const int j = w + G * t;                  // 0 .. 64*D*2*2/1024 - 1
      const bool isv = j >= NI * G / 2;
      const int jj = isv ? j - NI * G / 2 : j;
      const int row = jj * RPI + lane / CPR;    // this lane's row and LDS chunk position
      const int pos = lane % CPR;
      const int ch = isv ? pos : (pos ^ (row & (CPR - 1)));  // K: source-side XOR swizzle
      const uint32_t off = (bi * 64 + row < ctx) ? (uint32_t)((row * D + ch * 8) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(isv ? rv : rk, (da_lds_void*)(dst + (isv ? 64 * D : 0) + jj * 512),
                                               16, off, 0, 0, 0);
    }
  };

  // q stays bf16 (exact: it is the QKV GEMM's bf16 output) for the packed bf16 dot products; the softmax scale
  // is applied to the f32 score
  bf16_t* sQb = reinterpret_cast<bf16_t*>(sQ);
  // first block's DMA before the q prologue: its HBM latency overlaps the q / RoPE-table loads
  if (blk0 < blk1) stage(0, blk0);
  const int rpos = fused ? p.positions[b] : 0;
  // this step's k / v (fused path, last split) loaded now and consumed after the loop, so their latency is hidden
  const bool new_tok = fused && split == nsp - 1 && p.slots[b] >= 0;
  // QKV fold fused in: element col of this row = bf16(sum of the kg partial slabs (in slab order, as the fold
  // adds them) x the folded RMSNorm scale)
  // This lane's six elements (q halves, k halves, two v) and the row's sum of squares, four slabs per round with
  // every load issued before the first add (a dependent load-add chain per slab costs ~5 us per layer).
  const bool part = p.qkv_ws != nullptr;
  float pv[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (part) {
    const long pslab = (long)p.B * p.qkv_n;
    const int lq = lane & (D / 2 - 1), kcol = (p.Hq + hk) * D, vcol = (p.Hq + p.Hkv + hk) * D;
    const int col[6] = {hq * D + lq, hq * D + lq + D / 2, kcol + lq, kcol + lq + D / 2,
                        D == 128 ? vcol + 2 * lane : vcol + lane, D == 128 ? vcol + 2 * lane + 1 : vcol + lane};
    const float* row = p.qkv_ws + (long)b * p.qkv_n;
    const float* ssr = p.qkv_ws + (long)p.qkv_kg * pslab + b;
    for (int s0 = 0; s0 < p.qkv_kg; s0 += 4) {
      float t[4][7];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int sl = min(s0 + u, p.qkv_kg - 1);  // past the last slab: re-read it, dropped below
#pragma unroll
        for (int e = 0; e < 6; ++e) t[u][e] = row[(long)sl * pslab + col[e]];
        t[u][6] = ssr[(long)sl * p.B];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (s0 + u < p.qkv_kg) {
#pragma unroll
          for (int e = 0; e < 7; ++e) pv[e] += t[u][e];
        }
    }
    const float rstd = rsqrtf(pv[6] / p.qkv_k + p.qkv_eps);
#pragma unroll
    for (int e = 0; e < 6; ++e) pv[e] = bf2f(f2bf(pv[e] * rstd));
  }
  float kn0 = 0.f, kn1 = 0.f, kc0 = 0.f, ks0 = 0.f;
  uint32_t vn_pair = 0u;
  float vn_one = 0.f;
  if (new_tok) {
    const bf16_t* kn = p.knew + (long)b * p.new_bs + (long)hk * D;
    const bf16_t* vn = p.vnew + (long)b * p.new_bs + (long)hk * D;
    if (lane < D / 2) {
      kn0 = part ? pv[2] : bf2f(kn[lane]);
      kn1 = part ? pv[3] : bf2f(kn[lane + D / 2]);
      kc0 = p.rope_cos[(long)rpos * (D / 2) + lane];
      ks0 = p.rope_sin[(long)rpos * (D / 2) + lane];
    }
    if constexpr (D == 128) {
      vn_pair = part ? pack2(pv[4], pv[5])
                     : *reinterpret_cast<const uint32_t*>(vn + 2 * lane);
    } else {
      vn_one = part ? pv[4] : bf2f(vn[lane]);
    }
  }
  if (fused) {  // NeoX RoPE on q (f32 math, bf16 result: what rope_qkv_cache would have stored)
    const bf16_t* qs = p.q + (long)b * p.q_bs + (long)hq * D;
    const float* cp = p.rope_cos + (long)rpos * (D / 2);
    const float* sp = p.rope_sin + (long)rpos * (D / 2);
    for (int i = lane; i < D / 2; i += 64) {
      const float x0 = part ? pv[0] : bf2f(qs[i]);  // (i == lane: one pass)
      const float x1 = part ? pv[1] : bf2f(qs[i + D / 2]);
      const float c = cp[i], sn = sp[i];
      sQb[w * D + i] = f2bf(x0 * c - x1 * sn);
      sQb[w * D + i + D / 2] = f2bf(x1 * c + x0 * sn);
    }
  } else {
    for (int i = lane; i < D; i += 64) sQb[w * D + i] = p.q[(long)b * p.q_bs + (long)hq * D + i];
  }
  const float sl2 = p.scale * kLog2e;
  float m_run = -INFINITY, l_run = 0.f;
  float o0 = 0.f, o1 = 0.f;  // D=128: this lane's d = 2 lane, 2 lane + 1; D=64: d = lane
  // (no barrier here: each wave reads only its own sQ row; the loop's barrier publishes the ring)
  for (int bi = blk0, slot = 0; bi < blk1; ++bi, slot ^= 1) {
    if (bi + 1 < blk1) {
      stage(slot ^ 1, bi + 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");  // block bi landed, bi+1 in flight
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // raw barrier: __syncthreads' fence would drain the ring (vmcnt(0)) and serialise the prefetch
    __builtin_amdgcn_s_barrier();
    const bf16_t* sK = ring + slot * SLOT;
    const bf16_t* sV = sK + 64 * D;
    // lane = key
    const int key = bi * 64 + lane;
    // QK^T: 4 packed bf16 dot products (v_dot2c_f32_bf16) per 8-element chunk, two independent chains
    float sc0 = 0.f, sc1 = 0.f;
#pragma unroll
    for (int ch = 0; ch < CPR; ++ch) {
      // (pairs taken by shufflevector: bit-casting the elements of a uint32 x4 vector to bf16 x2 miscompiles
      // with this hipcc -- every pair reads element 0)
      const bf16x8d kv = __builtin_bit_cast(bf16x8d, *reinterpret_cast<const uint4_*>(sK + lane * D + ((ch ^ (lane & (CPR - 1))) << 3)));
      const bf16x8d qv = __builtin_bit_cast(bf16x8d, *reinterpret_cast<const uint4_*>(sQb + w * D + ch * 8));
      sc0 = __builtin_amdgcn_fdot2_f32_bf16(DA_PAIR(kv, 0), DA_PAIR(qv, 0), sc0, false);
      sc1 = __builtin_amdgcn_fdot2_f32_bf16(DA_PAIR(kv, 1), DA_PAIR(qv, 1), sc1, false);
      sc0 = __builtin_amdgcn_fdot2_f32_bf16(DA_PAIR(kv, 2), DA_PAIR(qv, 2), sc0, false);
      sc1 = __builtin_amdgcn_fdot2_f32_bf16(DA_PAIR(kv, 3), DA_PAIR(qv, 3), sc1, false);
    }
    float sc = (sc0 + sc1) * sl2;
    if (key >= ctx) sc = -INFINITY;
    const float mt = wave_max(sc);
    const float m_new = fmaxf(m_run, mt);
    const float alpha = exp2f(m_run - m_new);
    float e = key < ctx ? exp2f(sc - m_new) : 0.f;
    o0 *= alpha;
    o1 *= alpha;
    if constexpr (D == 128) {
      // P goes to LDS as bf16 and the denominator sums the same rounded values; P.V runs as packed bf16 dot
      // products over key pairs: v_perm gathers (V[k][d], V[k+1][d]) for this lane's two dims d
      const bf16_t eb = f2bf(e);
      e = bf2f(eb);
      l_run = l_run * alpha + wave_sum(e);
      m_run = m_new;
      bf16_t* sPb = reinterpret_cast<bf16_t*>(sP);
      sPb[w * 64 + lane] = eb;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's P row is written before it is read
      float a0 = 0.f, a1 = 0.f;
#pragma unroll 2
      for (int k = 0; k < 64; k += 8) {
        // P[k .. k+7] as 4 bf16 pairs
        const bf16x8d pk = __builtin_bit_cast(bf16x8d, *reinterpret_cast<const uint4_*>(sPb + w * 64 + k));
        auto pv = [&](int u, bf16x2d pp, float& c0, float& c1) {
          const uint32_t va = *reinterpret_cast<const uint32_t*>(sV + (k + 2 * u) * D + 2 * lane);
          const uint32_t vb = *reinterpret_cast<const uint32_t*>(sV + (k + 2 * u + 1) * D + 2 * lane);
          const uint32_t lo = __builtin_amdgcn_perm(vb, va, 0x05040100u);  // (V[k][2l],   V[k+1][2l])
          const uint32_t hi = __builtin_amdgcn_perm(vb, va, 0x07060302u);  // (V[k][2l+1], V[k+1][2l+1])
          c0 = __builtin_amdgcn_fdot2_f32_bf16(pp, __builtin_bit_cast(bf16x2d, lo), c0, false);
          c1 = __builtin_amdgcn_fdot2_f32_bf16(pp, __builtin_bit_cast(bf16x2d, hi), c1, false);
        };
        pv(0, DA_PAIR(pk, 0), o0, o1);
        pv(1, DA_PAIR(pk, 1), a0, a1);
        pv(2, DA_PAIR(pk, 2), o0, o1);
        pv(3, DA_PAIR(pk, 3), a0, a1);
      }
      o0 += a0;
      o1 += a1;
    } else {
      l_run = l_run * alpha + wave_sum(e);
      m_run = m_new;
      sP[w * 64 + lane] = e;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's sP row is written before it is read
#pragma unroll 4
      for (int k = 0; k < 64; k += 4) {
        const float4_ pk = *reinterpret_cast<const float4_*>(sP + w * 64 + k);
#pragma unroll
        for (int u = 0; u < 4; ++u) o0 += pk[u] * bf2f(sV[(k + u) * D + lane]);
      }
    }
    __builtin_amdgcn_s_barrier();  // every wave is done with this slot before it is refilled (block bi+2)
  }
  if (new_tok) {
    // this step's token: roped k (rounded to bf16, as the cache stores it) and v from the QKV rows, one more
    // online-softmax key; wave 0 writes both into the cache (no workgroup of this launch reads that row: the
    // block DMA range-checks it out)
    const int slot_new = p.slots[b];
    float kr0 = 0.f, kr1 = 0.f, part = 0.f;
    if (lane < D / 2) {
      const float x0 = kn0, x1 = kn1, c = kc0, sn = ks0;
      kr0 = bf2f(f2bf(x0 * c - x1 * sn));
      kr1 = bf2f(f2bf(x1 * c + x0 * sn));
      part = kr0 * bf2f(sQb[w * D + lane]) + kr1 * bf2f(sQb[w * D + lane + D / 2]);
    }
    const float sc = wave_sum(part) * sl2;
    const float m_new = fmaxf(m_run, sc);
    const float alpha = exp2f(m_run - m_new);
    float e = exp2f(sc - m_new);
    if constexpr (D == 128) e = bf2f(f2bf(e));  // P is bf16 on the cache path too
    l_run = l_run * alpha + e;
    m_run = m_new;
    if constexpr (D == 128) {
      o0 = o0 * alpha + e * bf2f(vn_pair & 0xffff);
      o1 = o1 * alpha + e * bf2f(vn_pair >> 16);
    } else {
      o0 = o0 * alpha + e * vn_one;
    }
    if (w == 0) {
      const long dst = (((long)(slot_new >> 6) * p.Hkv + hk) * 64 + (slot_new & 63)) * D;
      bf16_t* kc = const_cast<bf16_t*>(p.k_cache);
      bf16_t* vc = const_cast<bf16_t*>(p.v_cache);
      if (lane < D / 2) {
        kc[dst + lane] = f2bf(kr0);
        kc[dst + lane + D / 2] = f2bf(kr1);
      }
      // v from registers (the values attended above; bf16-exact)
      if constexpr (D == 128) *reinterpret_cast<uint32_t*>(vc + dst + 2 * lane) = vn_pair;
      else vc[dst + lane] = f2bf(vn_one);
    }
  }
  if (nsp == 1) {  // one split: normalise and write the output here (the combine skips this row)
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    bf16_t* op = p.o + (long)b * p.o_bs + (long)hq * D;
    if constexpr (D == 128) {
      *reinterpret_cast<uint32_t*>(op + 2 * lane) = pack2(o0 * inv, o1 * inv);
    } else {
      op[lane] = f2bf(o0 * inv);
    }
    return;
  }
  // partial results: ws[b][hq][split] = {m, l, o[D]}
  float* dst = p.ws + (((long)b * p.Hq + hq) * p.num_splits + split) * (D + 2);
  if (lane == 0) {
    dst[0] = m_run;
    dst[1] = l_run;
  }
  if constexpr (D == 128) {
    dst[2 + 2 * lane] = o0;
    dst[3 + 2 * lane] = o1;
  } else {
    dst[2 + lane] = o0;
  }
}

// Persistent form: a grid of about two workgroups per CU walks the (sequence, KV head, split) items, split
// fastest, so one long context's 8 x 64 split items land on 512 different workgroups while the empty items of
// short sequences (da_splits) cost a ctx_lens read each instead of a workgroup launch with 70 KB of LDS: a
// batch with one 64k-token sequence launched 16,384 workgroups per layer, 97 % of them empty, and the
// launch / LDS allocation of the empty ones took longer (1.17 ms per layer) than the attention itself.
template <int D, int NI>
__global__ void decode_attn_kernel(const DecodeAttnArgs p) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  const int total = p.B * p.Hkv * p.num_splits;
  const int S = p.num_splits;
  const bool rotate = (int)gridDim.x < total;  // persistent walk only (one workgroup per item needs no spreading)
  for (int item = blockIdx.x; item < total; item += gridDim.x) {
    // a sequence's splits sit at slots rotated by b: a short sequence's one real item lands on slot b % S instead
    // of slot 0, so the short sequences' items spread over the grid instead of piling onto the few workgroups
    // whose stride hits slot 0 (measured: 16 short sequences beside a 128k one made the launch 2.7x slower)
    const int sidx = item % S, r = item / S;
    const int b = r / p.Hkv, hk = r - b * p.Hkv;
    const int split = rotate ? (sidx - b % S + S) % S : sidx;
    decode_attn_item<D, NI>(p, dsm, b, hk, split);
    __syncthreads();  // the next item restages ring slot 0
  }
}

__global__ void decode_combine_kernel(const DecodeAttnArgs p) {
  const int b = blockIdx.x, hq = blockIdx.y;
  const int D = p.D;
  const int nsp = da_splits((p.ctx_lens[b] - (p.knew != nullptr ? 1 : 0) + 63) / 64, p.num_splits);
  if (nsp == 1) return;  // written by the attention workgroup itself
  const float* src = p.ws + ((long)b * p.Hq + hq) * p.num_splits * (D + 2);
  float m = -INFINITY;
  for (int s = 0; s < nsp; ++s) m = fmaxf(m, src[s * (D + 2)]);
  float l = 0.f;
  for (int s = 0; s < nsp; ++s) {
    const float ms = src[s * (D + 2)];
    if (ms != -INFINITY) l += src[s * (D + 2) + 1] * exp2f(ms - m);
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float acc = 0.f;
    for (int s = 0; s < nsp; ++s) {
      const float ms = src[s * (D + 2)];
      if (ms != -INFINITY) acc += src[s * (D + 2) + 2 + d] * exp2f(ms - m);
    }
    p.o[(long)b * p.o_bs + (long)hq * D + d] = f2bf(acc * inv);
  }
}

// ----------------------------------------------------------------------------
// Short-context decode attention, "wave per block" (D = 128, GQA group G = 4, one split).
// The split kernel above walks a (sequence, KV head)'s 64-token blocks one after another with ONE block in flight
// (two-slot ring), so at decode-batch contexts of a few hundred tokens its launch is mostly prologue and per-block
// HBM latency (B 64 x ctx 192: 18 us for 50 MB, 2.8 TB/s; gpurun_out/r6f_decode.log).  Here the G waves of the
// (sequence, KV head) workgroup each take their OWN blocks w, w + G, ... for ALL G query heads of the group (GQA:
// each K / V block is read once for the four heads), so the workgroup has G blocks (128 KB) in flight from its
// first instructions:
//  * K block by LDS-DMA into the wave's own 16 KB slot (source-side XOR swizzle: conflict-free lane = key reads);
//    V block straight into registers, 16 x buffer_load_dwordx4 (lane holds the 8-d chunk lane & 15 of the keys
//    (lane >> 4) + 4 j); both range-checked by the buffer descriptor (zero fill past the context);
//  * QK^T: lane = key, packed bf16 dot products against the G q rows (LDS broadcast reads);
//  * online softmax per head over the wave's blocks; P (bf16, the denominator sums the rounded values) through a
//    128-B LDS row per head, stored in the (key group, j) order the P.V step reads; P.V: v_perm key pairs + packed
//    bf16 dot products, 8 d per lane; the next block's K DMA is issued as soon as QK^T has read the slot, its V
//    loads as soon as P.V has consumed the registers;
//  * merge: the G waves' (m, l, o) partials meet in LDS (aliasing the K slots) and wave h combines head h with this
//    step's new token (roped k / v from the QKV rows or the QKV GEMM's split-K partials, attended from registers,
//    written to the cache by wave 0) -- the split kernel's prologue / new-token semantics, bit for bit in q, k, v.
// No wave waits for another before the merge: a wave's K slot and P rows are its own (its vmcnt / lgkmcnt cover
// them).  SHAI_DECODE_WB=0 / set_decode_wb(0) routes these launches back to the split kernel (A/B).
constexpr int kWbG = 4;
constexpr size_t kWbLds = (size_t)kWbG * 64 * 128 * 2 + (size_t)kWbG * 128 * 2 + (size_t)kWbG * kWbG * 64 * 2;

__global__ void __launch_bounds__(kWbG * 64, 2) decode_attn_wb_kernel(const DecodeAttnArgs p) {
  constexpr int G = kWbG, D = 128, CPR = D / 8;
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  bf16_t* sK = reinterpret_cast<bf16_t*>(dsm);   // [G waves][64 keys][D], swizzled
  bf16_t* sQb = sK + G * 64 * D;                 // [G heads][D]
  bf16_t* sPb = sQb + G * D;                     // [G waves][G heads][4 key groups][16]
  float* sM = reinterpret_cast<float*>(dsm);     // merge, aliasing the K slots: [G waves][G heads][2] (m, l)
  float* sO = sM + G * G * 2;                    // [G waves][G heads][4 key groups][D]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x / p.Hkv, hk = blockIdx.x - b * p.Hkv;
  const int hq = hk * G + w;  // this wave's head in the prologue and in the merge
  const bool fused = p.knew != nullptr;
  const int ctx = p.ctx_lens[b] - (fused ? 1 : 0);  // tokens read from the cache
  const int nblk = (ctx + 63) / 64;
  const int nmine = nblk > w ? (nblk - w + G - 1) / G : 0;  // blocks w, w + G, ... of this wave
  // physical ids of this wave's blocks, 64 per lane-distributed chunk (independent of ctx: issued beside its load)
  const int* bt = p.block_table + (long)b * p.max_blocks;
  int chunk0 = 0;
  int my_phys = (w + G * lane < p.max_blocks) ? bt[w + G * lane] : 0;
  auto phys_of = [&](int it) {
    if (it - chunk0 >= 64) {
      chunk0 += 64;
      const int e = w + G * (chunk0 + lane);
      my_phys = e < p.max_blocks ? bt[e] : 0;
    }
    return __builtin_amdgcn_readfirstlane(__shfl(my_phys, it - chunk0, 64));
  };
  const int lrow = lane >> 4, lpos = lane & 15;
  bf16_t* slot = sK + w * 64 * D;
  uint4_ vr[16];
  // descriptor sized to the block's rows inside the context: rows past it read as zeros (the range check of the
  // buffer instruction), so the offsets carry no per-lane select and fold into base + immediate / SGPR offsets
  auto rsrc = [&](const bf16_t* cache, int phys, int bi) {
    const int rows = min(64, ctx - bi * 64);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(cache + ((long)phys * p.Hkv + hk) * 64 * D),
                                             (short)0, rows * D * 2, 0x00020000);
  };
  // K: instruction t fills rows 4t .. 4t + 3 lane-linearly; LDS position lpos of row r holds global chunk
  // lpos ^ (r & 15), and (4t + lrow) & 15 repeats with t % 4
  int koff[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int row = 4 * t + lrow;
    koff[t] = (row * D + ((lpos ^ (row & (CPR - 1))) << 3)) * 2;
  }
  const int voff = (lrow * D + lpos * 8) * 2;  // V: row lrow + 4 j at voff + 1024 j
  auto issue_k = [&](int bi, int phys) {
    const __amdgpu_buffer_rsrc_t rk = rsrc(p.k_cache, phys, bi);
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      SHAI_DASSERT_DMA(koff[t & 3] + (t >> 2) * 4096, 64 * D * 2, 0x80000000u);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (da_lds_void*)(slot + t * 512), 16, koff[t & 3], (t >> 2) * 4096,
                                               0, 0);
    }
  };
  auto issue_v = [&](int bi, int phys) {
    const __amdgpu_buffer_rsrc_t rv = rsrc(p.v_cache, phys, bi);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      SHAI_DASSERT_DMA(voff + j * 1024, 64 * D * 2, 0x80000000u);
      vr[j] = __builtin_bit_cast(
          uint4_, __builtin_amdgcn_raw_buffer_load_b128(rv, voff + (j & 3) * 1024, (j >> 2) * 4096, 0));
    }
  };
  if (nmine > 0) {
    const int ph = phys_of(0);
    issue_k(w, ph);
    issue_v(w, ph);
  }

  // ---- prologue (as the split kernel): this wave's q head, roped, into sQb; the new token's k / v in registers
  const int rpos = fused ? p.positions[b] : 0;
  const bool new_tok = fused && p.slots[b] >= 0;
  const bool part = p.qkv_ws != nullptr;
  float pv[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (part) {
    const long pslab = (long)p.B * p.qkv_n;
    const int lq = lane & (D / 2 - 1), kcol = (p.Hq + hk) * D, vcol = (p.Hq + p.Hkv + hk) * D;
    const int col[6] = {hq * D + lq, hq * D + lq + D / 2, kcol + lq, kcol + lq + D / 2, vcol + 2 * lane,
                        vcol + 2 * lane + 1};
    const float* row = p.qkv_ws + (long)b * p.qkv_n;
    const float* ssr = p.qkv_ws + (long)p.qkv_kg * pslab + b;
    for (int s0 = 0; s0 < p.qkv_kg; s0 += 4) {
      float t[4][7];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int sl = min(s0 + u, p.qkv_kg - 1);
#pragma unroll
        for (int e = 0; e < 6; ++e) t[u][e] = row[(long)sl * pslab + col[e]];
        t[u][6] = ssr[(long)sl * p.B];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (s0 + u < p.qkv_kg) {
#pragma unroll
          for (int e = 0; e < 7; ++e) pv[e] += t[u][e];
        }
    }
    const float rstd = rsqrtf(pv[6] / p.qkv_k + p.qkv_eps);
#pragma unroll
    for (int e = 0; e < 6; ++e) pv[e] = bf2f(f2bf(pv[e] * rstd));
  }
  float kn0 = 0.f, kn1 = 0.f, kc0 = 0.f, ks0 = 0.f;
  uint32_t vn_pair = 0u;
  if (new_tok) {
    const bf16_t* kn = p.knew + (long)b * p.new_bs + (long)hk * D;
    const bf16_t* vn = p.vnew + (long)b * p.new_bs + (long)hk * D;
    kn0 = part ? pv[2] : bf2f(kn[lane]);
    kn1 = part ? pv[3] : bf2f(kn[lane + D / 2]);
    kc0 = p.rope_cos[(long)rpos * (D / 2) + lane];
    ks0 = p.rope_sin[(long)rpos * (D / 2) + lane];
    vn_pair = part ? pack2(pv[4], pv[5]) : *reinterpret_cast<const uint32_t*>(vn + 2 * lane);
  }
  if (fused) {  // NeoX RoPE on q (f32 math, bf16 result), lane = rotation pair (D / 2 = 64)
    const bf16_t* qs = p.q + (long)b * p.q_bs + (long)hq * D;
    const float x0 = part ? pv[0] : bf2f(qs[lane]);
    const float x1 = part ? pv[1] : bf2f(qs[lane + D / 2]);
    const float c = p.rope_cos[(long)rpos * (D / 2) + lane], sn = p.rope_sin[(long)rpos * (D / 2) + lane];
    sQb[w * D + lane] = f2bf(x0 * c - x1 * sn);
    sQb[w * D + lane + D / 2] = f2bf(x1 * c + x0 * sn);
  } else {
    const bf16_t* qs = p.q + (long)b * p.q_bs + (long)hq * D;
    *reinterpret_cast<uint32_t*>(sQb + w * D + 2 * lane) = *reinterpret_cast<const uint32_t*>(qs + 2 * lane);
  }
  // every wave reads all G q rows: raw barrier (a __syncthreads fence would drain the K / V loads in flight)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  const float sl2 = p.scale * kLog2e;
  float m_run[G], l_run[G], o[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    m_run[h] = -INFINITY;
    l_run[h] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[h][i] = 0.f;
  }
  bf16_t* sPw = sPb + w * G * 64;
  for (int it = 0; it < nmine; ++it) {
    const int bi = w + G * it;
    // this block's K slot has landed (its V loads, issued behind it, may still be in flight)
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    // ---- S = q K^T for the G heads, lane = key
    float a0[G], a1[G];
#pragma unroll
    for (int h = 0; h < G; ++h) a0[h] = a1[h] = 0.f;
#pragma unroll 2
    for (int ch = 0; ch < CPR; ++ch) {
      const bf16x8d kv =
          __builtin_bit_cast(bf16x8d, *reinterpret_cast<const uint4_*>(slot + lane * D + ((ch ^ (lane & (CPR - 1))) << 3)));
#pragma unroll
      for (int h = 0; h < G; ++h) {
        const bf16x8d qv = __builtin_bit_cast(bf16x8d, *reinterpret_cast<const uint4_*>(sQb + h * D + ch * 8));
        a0[h] = __builtin_amdgcn_fdot2_f32_bf16(DA_PAIR(kv, 0), DA_PAIR(qv, 0), a0[h], false);
        a1[h] = __builtin_amdgcn_fdot2_f32_bf16(DA_PAIR(kv, 1), DA_PAIR(qv, 1), a1[h], false);
        a0[h] = __builtin_amdgcn_fdot2_f32_bf16(DA_PAIR(kv, 2), DA_PAIR(qv, 2), a0[h], false);
        a1[h] = __builtin_amdgcn_fdot2_f32_bf16(DA_PAIR(kv, 3), DA_PAIR(qv, 3), a1[h], false);
      }
    }
    // the K slot is read: the next block's K DMA goes out now (its phys id comes from the read-ahead chunk)
    const bool more = it + 1 < nmine;
    int ph_next = 0;
    if (more) {
      ph_next = phys_of(it + 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue_k(bi + G, ph_next);
    }
    // ---- online softmax per head; P row (bf16) in (key group, j) order: key = g + 4 j -> [g][j]
    const int key = bi * 64 + lane;
    const bool valid = key < ctx;
#pragma unroll
    for (int h = 0; h < G; ++h) {
      const float s = valid ? (a0[h] + a1[h]) * sl2 : -INFINITY;
      const float m_new = fmaxf(m_run[h], wave_max(s));  // the block holds >= 1 valid key: finite
      const float alpha = exp2f(m_run[h] - m_new);
      const bf16_t eb = f2bf(valid ? exp2f(s - m_new) : 0.f);
      l_run[h] = l_run[h] * alpha + wave_sum(bf2f(eb));
      m_run[h] = m_new;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[h][i] *= alpha;
      sPw[h * 64 + (lane & 3) * 16 + (lane >> 2)] = eb;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's P rows are written before they are read
    // ---- O += P V: lane group g = lane >> 4 owns keys g + 4 j (j = 0..15), d = 8 lpos .. 8 lpos + 7
    uint32_t pp[G][8];
#pragma unroll
    for (int h = 0; h < G; ++h) {
      const uint4_ pa = *reinterpret_cast<const uint4_*>(sPw + h * 64 + lrow * 16);
      const uint4_ pb = *reinterpret_cast<const uint4_*>(sPw + h * 64 + lrow * 16 + 8);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pp[h][i] = pa[i];
        pp[h][4 + i] = pb[i];
      }
    }
#pragma unroll
    for (int jp = 0; jp < 8; ++jp) {  // keys (2 jp, 2 jp + 1) of the group: P pair pp[h][jp]
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t va = vr[2 * jp][i], vb = vr[2 * jp + 1][i];
        const bf16x2d lo = __builtin_bit_cast(bf16x2d, __builtin_amdgcn_perm(vb, va, 0x05040100u));  // d = 2i
        const bf16x2d hi = __builtin_bit_cast(bf16x2d, __builtin_amdgcn_perm(vb, va, 0x07060302u));  // d = 2i + 1
#pragma unroll
        for (int h = 0; h < G; ++h) {
          const bf16x2d pk = __builtin_bit_cast(bf16x2d, pp[h][jp]);
          o[h][2 * i] = __builtin_amdgcn_fdot2_f32_bf16(pk, lo, o[h][2 * i], false);
          o[h][2 * i + 1] = __builtin_amdgcn_fdot2_f32_bf16(pk, hi, o[h][2 * i + 1], false);
        }
      }
    }
    // (no scheduling across: hoisting the next block's V loads above P.V would need a second 64-register set)
    __builtin_amdgcn_sched_barrier(0);
    if (more) issue_v(bi + G, ph_next);
  }

  // ---- merge the G waves' partials (the buffers alias the K slots: every wave is past its last QK^T read)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int h = 0; h < G; ++h) {
      sM[(w * G + h) * 2] = m_run[h];
      sM[(w * G + h) * 2 + 1] = l_run[h];
    }
  }
#pragma unroll
  for (int h = 0; h < G; ++h) {
    float* dst = sO + ((w * G + h) * 4 + lrow) * D + lpos * 8;
    *reinterpret_cast<float4_*>(dst) = float4_{o[h][0], o[h][1], o[h][2], o[h][3]};
    *reinterpret_cast<float4_*>(dst + 4) = float4_{o[h][4], o[h][5], o[h][6], o[h][7]};
  }
  __syncthreads();
  // wave w: head hq; lane holds d = 2 lane, 2 lane + 1
  float s_new = -INFINITY, kr0 = 0.f, kr1 = 0.f;
  if (new_tok) {
    kr0 = bf2f(f2bf(kn0 * kc0 - kn1 * ks0));  // roped k, rounded to bf16 as the cache stores it
    kr1 = bf2f(f2bf(kn1 * kc0 + kn0 * ks0));
    s_new = wave_sum(kr0 * bf2f(sQb[w * D + lane]) + kr1 * bf2f(sQb[w * D + lane + D / 2])) * sl2;
  }
  float M = s_new;
#pragma unroll
  for (int ww = 0; ww < G; ++ww) M = fmaxf(M, sM[(ww * G + w) * 2]);
  float L = 0.f, o0 = 0.f, o1 = 0.f;
#pragma unroll
  for (int ww = 0; ww < G; ++ww) {
    const float mw = sM[(ww * G + w) * 2];
    const float f = mw == -INFINITY ? 0.f : exp2f(mw - M);
    L += sM[(ww * G + w) * 2 + 1] * f;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float2 v = *reinterpret_cast<const float2*>(sO + ((ww * G + w) * 4 + g) * D + 2 * lane);
      o0 += v.x * f;
      o1 += v.y * f;
    }
  }
  if (new_tok) {
    const float e = bf2f(f2bf(exp2f(s_new - M)));  // P is bf16 on the cache path too
    L += e;
    o0 += e * bf2f(vn_pair & 0xffff);
    o1 += e * bf2f(vn_pair >> 16);
    if (w == 0) {  // this step's k / v into the cache (no workgroup of this launch reads that row)
      const int slot_new = p.slots[b];
      const long dst = (((long)(slot_new >> 6) * p.Hkv + hk) * 64 + (slot_new & 63)) * D;
      bf16_t* kc = const_cast<bf16_t*>(p.k_cache);
      bf16_t* vc = const_cast<bf16_t*>(p.v_cache);
      kc[dst + lane] = f2bf(kr0);
      kc[dst + lane + D / 2] = f2bf(kr1);
      *reinterpret_cast<uint32_t*>(vc + dst + 2 * lane) = vn_pair;
    }
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  *reinterpret_cast<uint32_t*>(p.o + (long)b * p.o_bs + (long)hq * D + 2 * lane) = pack2(o0 * inv, o1 * inv);
}

static int g_decode_wb = -1;
int decode_wb_mode() {
  if (g_decode_wb < 0) {
    const char* e = getenv("SHAI_DECODE_WB");
    g_decode_wb = (e != nullptr && atoi(e) == 0) ? 0 : 1;
  }
  return g_decode_wb;
}
int set_decode_wb(int mode) {
  const int prev = decode_wb_mode();
  if (mode >= 0) g_decode_wb = mode;
  return prev;
}

size_t decode_attn_workspace(int B, int Hq, int D, int num_splits) {
  return (size_t)B * Hq * num_splits * (D + 2) * sizeof(float);
}

void launch_decode_attn(const DecodeAttnArgs& a, hipStream_t s) {
  const int G = a.Hq / a.Hkv;
  if (a.D == 128 && G == kWbG && a.num_splits == 1 && decode_wb_mode()) {  // wave-per-block short-context kernel
    decode_attn_wb_kernel<<<dim3((unsigned)(a.B * a.Hkv)), kWbG * 64, kWbLds, s>>>(a);
    return;
  }
  static const int width = [] {  // two workgroups per CU (70 KB of LDS each)
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
    return 2 * cus;
  }();
  // short-context batches (<= 8 splits: every item does work) keep one workgroup per item; the persistent walk is
  // for the raised split factors of long contexts.  SHAI_DECODE_PERSIST=0 / 1 forces either form (A/B).
  static const int force = [] {
    const char* e = getenv("SHAI_DECODE_PERSIST");
    return e ? (e[0] == '1' ? 1 : 0) : -1;
  }();
  const long items = (long)a.B * a.Hkv * a.num_splits;
  const bool persist = force >= 0 ? force == 1 : a.num_splits > 8;
  dim3 grid((unsigned)(persist ? std::min<long>(items, width) : items));
  const size_t lds = (size_t)4 * 64 * a.D * sizeof(bf16_t) + (size_t)8 * a.D * 4 + 8 * 64 * 4;
  // NI = wave DMA instructions per block per wave = (2 * 64 * D * 2 / 1024) / G
#define DA(D_, NI_) decode_attn_kernel<D_, NI_><<<grid, G * 64, lds, s>>>(a)
  if (a.D == 128) {
    switch (G) {
      case 1: DA(128, 32); break;
      case 2: DA(128, 16); break;
      case 4: DA(128, 8); break;
      default: DA(128, 4); break;  // G = 8
    }
  } else {
    switch (G) {
      case 1: DA(64, 16); break;
      case 2: DA(64, 8); break;
      case 4: DA(64, 4); break;
      default: DA(64, 2); break;
    }
  }
#undef DA
  if (a.num_splits > 1) decode_combine_kernel<<<dim3(a.B, a.Hq), 128, 0, s>>>(a);
}

// ----------------------------------------------------------------------------
// KV cache write: cache layout [num_blocks, Hkv, 64, D]; slot = block*64 + off
// ----------------------------------------------------------------------------
__global__ void kv_write_kernel(const bf16_t* __restrict__ k, const bf16_t* __restrict__ v, bf16_t* __restrict__ kc,
                                bf16_t* __restrict__ vc, const int* __restrict__ slots, int T, int Hkv, int D,
                                long k_ts, long v_ts) {
  const int CPR = D / 8;
  const long total = (long)T * Hkv * CPR;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % CPR);
    const int h = (int)((i / CPR) % Hkv);
    const int t = (int)(i / ((long)CPR * Hkv));
    const int slot = slots[t];
    if (slot < 0) continue;
    const long dst = (((long)(slot >> 6) * Hkv + h) * 64 + (slot & 63)) * D + ch * 8;
    *reinterpret_cast<uint4_*>(kc + dst) = *reinterpret_cast<const uint4_*>(k + (long)t * k_ts + (long)h * D + ch * 8);
    *reinterpret_cast<uint4_*>(vc + dst) = *reinterpret_cast<const uint4_*>(v + (long)t * v_ts + (long)h * D + ch * 8);
  }
}

void launch_kv_write(const bf16_t* k, const bf16_t* v, bf16_t* k_cache, bf16_t* v_cache, const int* slot_mapping, int T,
                     int Hkv, int D, long k_ts, long v_ts, hipStream_t s) {
  const long total = (long)T * Hkv * (D / 8);
  long blocks = (total + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  kv_write_kernel<<<(int)blocks, 256, 0, s>>>(k, v, k_cache, v_cache, slot_mapping, T, Hkv, D, k_ts, v_ts);
}

// Fused decode/prefill prologue on the packed QKV projection [T, (H + 2 Hkv) * D] (row stride ld):
// NeoX RoPE on q (in place) and k, then k and v scattered into the paged caches [blocks, Hkv, 64, D].
// One item = 16 elements: for q/k heads, 8 elements of each rotation half; for v heads, a 16-element
// copy.  Replaces rope(q) + rope(k) + kv_write (3 launches and an extra pass over k).
__global__ void rope_qkv_cache_kernel(bf16_t* __restrict__ qkv, long ld, const int* __restrict__ pos,
                                      const float* __restrict__ cs, const float* __restrict__ sn,
                                      bf16_t* __restrict__ kc, bf16_t* __restrict__ vc, const int* __restrict__ slots,
                                      int T, int H, int Hkv, int D) {
  const int half = D >> 1;
  const int per_head = D / 16;
  const int heads = H + 2 * Hkv;
  const long total = (long)T * heads * per_head;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % per_head);
    const int hh = (int)((i / per_head) % heads);
    const int t = (int)(i / ((long)per_head * heads));
    bf16_t* row = qkv + (long)t * ld;
    const int slot = slots[t];
    if (hh >= H + Hkv) {  // v head: copy 16 elements
      if (slot < 0) continue;
      const int h = hh - H - Hkv;
      const bf16_t* src = row + (long)hh * D + c * 16;
      const long dst = (((long)(slot >> 6) * Hkv + h) * 64 + (slot & 63)) * D + c * 16;
      *reinterpret_cast<uint4_*>(vc + dst) = *reinterpret_cast<const uint4_*>(src);
      *reinterpret_cast<uint4_*>(vc + dst + 8) = *reinterpret_cast<const uint4_*>(src + 8);
      continue;
    }
    bf16_t* xh = row + (long)hh * D;
    const int p = pos[t];
    float a[8], b[8];
    unpack8(*reinterpret_cast<const uint4_*>(xh + 8 * c), a);
    unpack8(*reinterpret_cast<const uint4_*>(xh + half + 8 * c), b);
    const float* cp = cs + (long)p * half + 8 * c;
    const float* sp = sn + (long)p * half + 8 * c;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float co = cp[e], si = sp[e];
      const float x0 = a[e], x1 = b[e];
      a[e] = x0 * co - x1 * si;
      b[e] = x1 * co + x0 * si;
    }
    const uint4_ ua = pack8(a), ub = pack8(b);
    if (hh < H) {
      *reinterpret_cast<uint4_*>(xh + 8 * c) = ua;
      *reinterpret_cast<uint4_*>(xh + half + 8 * c) = ub;
    } else if (slot >= 0) {
      const int h = hh - H;
      const long dst = (((long)(slot >> 6) * Hkv + h) * 64 + (slot & 63)) * D;
      *reinterpret_cast<uint4_*>(kc + dst + 8 * c) = ua;
      *reinterpret_cast<uint4_*>(kc + dst + half + 8 * c) = ub;
    }
  }
}

void launch_rope_qkv_cache(bf16_t* qkv, long ld, const int* pos, const float* cos, const float* sin, bf16_t* k_cache,
                           bf16_t* v_cache, const int* slots, int T, int H, int Hkv, int D, hipStream_t s) {
  const long total = (long)T * (H + 2 * Hkv) * (D / 16);
  long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  rope_qkv_cache_kernel<<<(int)blocks, 256, 0, s>>>(qkv, ld, pos, cos, sin, k_cache, v_cache, slots, T, H, Hkv, D);
}

}  // namespace shai
