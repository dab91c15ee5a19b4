// bf16 GEMM, v5 "four big waves": 256 x 256 output tile, 4 waves of 128 x 128 each, one wave per SIMD.
//
//   C[m, n] = act(alpha * sum_k A[m, k] * W[n, k] + bias[n]) + res_alpha * R[m, n]
//
// Why: the v4 kernel (gemm_8ph.hip) pairs two waves per SIMD that each own a 128 x 64 (or 128 x 80) slice;
// per 64-deep K-tile a CU then reads 8 x (128 + 80) x 128 B = 213 KB of fragments out of LDS and re-syncs
// all 8 waves at 8 barriers, and it stalls at 45-58 % MFMA busy (profiles/pmc_round3.md) -- the level of the
// 8-phase template.  A 128 x 128 wave tile reads 4 x 256 x 128 B = 131 KB per K-tile (-38 %) and needs one
// barrier per K-tile; with 256 accumulator registers a wave owns its SIMD, so it hides its own LDS latency by
// software pipelining instead of a partner wave:
//
// * LDS: 2 stages of (A 256 x 64 | W 256 x 64) bf16 = 128 KB, filled by LDS-DMA (`buffer_load ... lds`,
//   16 B per lane, 8 rows x 128 B per wave-instruction, 16 per wave per K-tile), rows swizzled as in v4
//   (16-B chunk ^= (row >> 1) & 7 on the source address and on the read): conflict-free ds_read_b128.
// * Fragments double-buffered in registers (2 sets x (8 X + 8 W) x 4 VGPRs): per K-tile t
//     (a) MFMAs of k-step 0 (fragment set 0) interleaved with the ds_reads of k-step 1 (set 1);
//     (b) lgkmcnt(0) + vmcnt(0) (this wave's DMA of tile t+1 landed) + ONE s_barrier;
//     (c) MFMAs of k-step 1 (set 1) interleaved with the DMA of tile t+2 into the stage tile t just vacated
//         and the ds_reads of tile t+1's k-step 0 (set 0).
//   The barrier in (b) is both the RAW fence for tile t+1 (every wave's DMA retired before it) and the WAR
//   fence for tile t's stage (every wave's reads of it retired by the lgkmcnt(0) before it).
// * `sched_group_barrier` pins the interleave: 2 ds_reads (+ 2 DMA in (c)) per 8 MFMAs.
// * Each lane stores 8 consecutive columns with one 16-B store: the W tile is staged with its rows permuted
//   inside pairs of 16-column MFMA blocks (as v4's wide epilogue).
// * XCD-aware bijective block remap + grouped M ordering (v4).
#include "gemm_epilogue.h"

#include <type_traits>

namespace shai {

typedef __bf16 w4bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void w4_lds_void;

constexpr int W4_BM = 256, W4_BN = 256, W4_BK = 64;
constexpr int W4_STAGE = (W4_BM + W4_BN) * W4_BK;  // elements per LDS stage (64 KB)
constexpr uint32_t W4_OOB = 0x80000000u;

__device__ __forceinline__ int w4_swz(int row, int ch) { return row * W4_BK + ((ch ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t w4_rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)min(bytes, 0x7fffffffL),
                                           0x00020000);
}

// W-tile LDS row r (0..255) -> tile-local output column: rows permuted inside each pair of 16-column blocks of
// a wave's 128 columns so that lane quad fq of the block pair (2q, 2q+1) owns columns 32q + 8fq .. + 7.
__device__ __forceinline__ int w4_wperm(int r) {
  const int g = r >> 7, loc = r & 127;
  const int jb = loc >> 4, nn = loc & 15;
  return g * 128 + (jb >> 1) * 32 + (nn >> 2) * 8 + (jb & 1) * 4 + (nn & 3);
}

template <int ACT, bool GLU>
__global__ void __launch_bounds__(256, 1) gemm_w4_kernel(const GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) bf16_t w4_smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  // ---- tile mapping: XCD remap (bijective) + grouped M ordering
  const int tiles_m = (p.M + W4_BM - 1) / W4_BM, tiles_n = (p.N + W4_BN - 1) / W4_BN;
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
  const int m0 = (first_m + in_group % gsize) * W4_BM;
  const int n0 = (in_group / gsize) * W4_BN;

  const __amdgpu_buffer_rsrc_t rA = w4_rsrc(p.A, (long)p.M * p.lda * 2);
  const __amdgpu_buffer_rsrc_t rW = w4_rsrc(p.W, (long)p.N * p.ldw * 2);

  // ---- DMA geometry: wave wid stages rows wid*64 + j*8 + lrow (j < 8) of A and of W; the lane's 16-B source
  // chunk is the swizzled one, the LDS image lane-linear.  Invalid rows carry the OOB bit (zero fill).
  const int lrow = lane >> 3, lpos = lane & 7;
  uint32_t aoff[8], woff[8];
  // source chunk landing at position lpos of LDS row r: lpos ^ ((r >> 1) & 7) = lpos ^ (lrow >> 1) ^ 4 (j & 1)
  const int kch0 = (lpos ^ (lrow >> 1)) * 8, kch1 = (lpos ^ (lrow >> 1) ^ 4) * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r = wid * 64 + j * 8 + lrow;         // LDS row (A and W alike)
    const int ch = lpos ^ ((r >> 1) & 7);
    const int m = m0 + r;
    aoff[j] = m < p.M ? (uint32_t)(((long)m * p.lda + ch * 8) * 2) : W4_OOB;
    const int n = n0 + w4_wperm(r);
    woff[j] = n < p.N ? (uint32_t)(((long)n * p.ldw + ch * 8) * 2) : W4_OOB;
  }
  const int nk = (p.K + W4_BK - 1) / W4_BK;
  // g < 8: A rows j = g; g >= 8: W rows j = g - 8.  Ragged last K-tile: chunks past K read zero.
  auto dma = [&](int stage, int t, int g) {
    bf16_t* base = w4_smem + stage * W4_STAGE;
    const int k0 = t * W4_BK;
    const bool oob_k = k0 + ((g & 1) ? kch1 : kch0) >= p.K;   // row j = g & 7: parity of j = parity of g
    if (g < 8) {
      const uint32_t off = oob_k ? W4_OOB : aoff[g] + (uint32_t)k0 * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (w4_lds_void*)(base + (wid * 64 + g * 8) * W4_BK), 16, off, 0, 0,
                                               0);
    } else {
      const uint32_t off = oob_k ? W4_OOB : woff[g - 8] + (uint32_t)k0 * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (w4_lds_void*)(base + W4_BM * W4_BK + (wid * 64 + (g - 8) * 8) *
                                                                                             W4_BK),
                                               16, off, 0, 0, 0);
    }
  };

  // ---- fragment reads: row (wr*128 | wc*128) + 16 i + fr, chunk 4 ks + fq; the swizzle depends on fr only
  const int fr = lane & 15, fq = lane >> 4;
  // element offset of fragment (i, ks) inside a stage (A part): (wr*128 + 16 i + fr) * 64 + swizzled chunk
  auto xoff = [&](int i, int ks) { return (wr * 128 + 16 * i + fr) * W4_BK + (((fq + 4 * ks) ^ ((fr >> 1) & 7)) << 3); };
  auto woffl = [&](int j, int ks) {
    return W4_BM * W4_BK + (wc * 128 + 16 * j + fr) * W4_BK + (((fq + 4 * ks) ^ ((fr >> 1) & 7)) << 3);
  };

  // Accumulators start life as the first k-step's MFMAs with an inline-zero C operand: zero-initialising
  // 64 loop-carried accumulators makes hipcc shuffle them between AGPRs inside the loop (~100-400
  // v_accvgpr moves per K-tile); with distinct first values they stay in place.
  float4_ acc[8][8];
  w4bf16x8 x0[8], w0[8], x1[8], w1[8];

  // ---- prologue: tiles 0 and 1 in flight, wait for tile 0, k-step 0 fragments of tile 0
#pragma unroll
  for (int g = 0; g < 16; ++g) dma(0, 0, g);
#pragma unroll
  for (int g = 0; g < 16; ++g) dma(1, 1, g);   // nk == 1: zero fill past K, never read
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 8; ++i) x0[i] = *reinterpret_cast<const w4bf16x8*>(w4_smem + xoff(i, 0));
#pragma unroll
  for (int j = 0; j < 8; ++j) w0[j] = *reinterpret_cast<const w4bf16x8*>(w4_smem + woffl(j, 0));

  // (a) k-step 0 MFMAs of tile t (set 0) || reads of its k-step 1 (set 1), W fragments first (the first MFMA
  // group of (c) needs all of them), 4 reads per 8 MFMAs over the first 4 groups.  FIRST: C = 0.
  auto seg_a = [&](int t, auto first_t) {
    constexpr bool FIRST = decltype(first_t)::value;
    const bf16_t* sc = w4_smem + (t & 1) * W4_STAGE;
    const float4_ z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      if (g < 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int f = 4 * g + u;  // 0..15: w1[0..7], x1[0..7]
          if (f < 8) w1[f] = *reinterpret_cast<const w4bf16x8*>(sc + woffl(f, 1));
          else x1[f - 8] = *reinterpret_cast<const w4bf16x8*>(sc + xoff(f - 8, 1));
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[j], x0[g], FIRST ? z : acc[g][j], 0, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      if (g < 4) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  // (b) this wave's reads of stage t and its DMA of tile t+1 retired; one barrier for all four waves.  The
  // empty asm redefines set 1 after the wait: hipcc's own waitcnt pass does not see the inline wait and would
  // otherwise hold (c)'s MFMAs for the set-0 reads issued there.
  // (c) k-step 1 MFMAs (set 1) || DMA of tile t+2 into the vacated stage (2 per 8 MFMAs; past K it is a zero
  // fill nobody reads) || reads of tile t+1's k-step 0 (set 0, W first) over the first 4 groups; then the
  // same inline-wait trick for set 0 (its reads are long done by the segment's end).
  auto seg_bc = [&](int t) {
    const int c = t & 1;
    const bf16_t* sn = w4_smem + (c ^ 1) * W4_STAGE;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int g = 0; g < 8; ++g) asm volatile("" : "+v"(x1[g]), "+v"(w1[g]));
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      dma(c, t + 2, g);
      dma(c, t + 2, g + 8);
      if (g < 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int f = 4 * g + u;
          if (f < 8) w0[f] = *reinterpret_cast<const w4bf16x8*>(sn + woffl(f, 0));
          else x0[f - 8] = *reinterpret_cast<const w4bf16x8*>(sn + xoff(f - 8, 0));
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[j], x1[g], acc[g][j], 0, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
      if (g < 4) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int g = 0; g < 8; ++g) asm volatile("" : "+v"(x0[g]), "+v"(w0[g]));
  };

  seg_a(0, std::true_type{});
  for (int t = 0; t + 1 < nk; ++t) {
    seg_bc(t);
    seg_a(t + 1, std::false_type{});
  }
  seg_bc(nk - 1);

  // ---- epilogue: lane owns row m0 + wr*128 + 16 i + fr, columns n0 + wc*128 + 32 q + 8 fq .. + 7 (q < 4)
  bf16_t* C = p.C;
  const bf16_t* R = p.residual;
  const bool full = m0 + W4_BM <= p.M && n0 + W4_BN <= p.N && ((p.ldc | (R ? p.ldr : 0)) & 7) == 0 &&
                    ((((uintptr_t)C) | (uintptr_t)R | (uintptr_t)p.bias) & 15) == 0;
  if (full) {
    float bq[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (p.bias) unpack8(*reinterpret_cast<const uint4_*>(p.bias + n0 + wc * 128 + q * 32 + 8 * fq), bq[q]);
      else
#pragma unroll
        for (int e = 0; e < 8; ++e) bq[q][e] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const long m = m0 + wr * 128 + 16 * i + fr;
      uint4_ rr[4];
      if (!GLU && R) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          rr[q] = *reinterpret_cast<const uint4_*>(R + m * p.ldr + n0 + wc * 128 + q * 32 + 8 * fq);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[i][2 * q][e] * p.alpha + bq[q][e];
          v[4 + e] = acc[i][2 * q + 1][e] * p.alpha + bq[q][4 + e];
        }
        if constexpr (GLU) {  // (value, gate) column pairs: the lane's 8 columns give 4 consecutive outputs
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = v[2 * e] * apply_act<ACT>(v[2 * e + 1]);
          if (R) {
            const uint2_ r2 = *reinterpret_cast<const uint2_*>(R + m * p.ldr + ((n0 + wc * 128 + q * 32 + 8 * fq) >> 1));
            o[0] += bf2f(r2[0] & 0xffff) * p.res_alpha; o[1] += bf2f(r2[0] >> 16) * p.res_alpha;
            o[2] += bf2f(r2[1] & 0xffff) * p.res_alpha; o[3] += bf2f(r2[1] >> 16) * p.res_alpha;
          }
          uint2_ w;
          w[0] = pack2(o[0], o[1]);
          w[1] = pack2(o[2], o[3]);
          *reinterpret_cast<uint2_*>(C + m * p.ldc + ((n0 + wc * 128 + q * 32 + 8 * fq) >> 1)) = w;
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = apply_act<ACT>(v[e]);
          if (R) {
            float r8[8];
            unpack8(rr[q], r8);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += r8[e] * p.res_alpha;
          }
          *reinterpret_cast<uint4_*>(C + m * p.ldc + n0 + wc * 128 + q * 32 + 8 * fq) = pack8(v);
        }
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wr * 128 + 16 * i + fr;
#pragma unroll
      for (int jb = 0; jb < 8; ++jb) {
        const int n = n0 + wc * 128 + (jb >> 1) * 32 + 8 * fq + 4 * (jb & 1);
        if constexpr (GLU) {  // edge tiles: guarded (value, gate) pairs
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            if (m < p.M && n + e + 1 < p.N) {
              const float a = acc[i][jb][e] * p.alpha + (p.bias ? bf2f(p.bias[n + e]) : 0.f);
              const float gt = acc[i][jb][e + 1] * p.alpha + (p.bias ? bf2f(p.bias[n + e + 1]) : 0.f);
              float v = a * apply_act<ACT>(gt);
              const int nc = (n + e) >> 1;
              if (R) v += bf2f(R[(long)m * p.ldr + nc]) * p.res_alpha;
              C[(long)m * p.ldc + nc] = f2bf(v);
            }
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {   // edge tiles: element-wise, guarded (no array indexed at run time)
            if (m < p.M && n + e < p.N) {
              float v = apply_act<ACT>(acc[i][jb][e] * p.alpha + (p.bias ? bf2f(p.bias[n + e]) : 0.f));
              if (R) v += bf2f(R[(long)m * p.ldr + n + e]) * p.res_alpha;
              C[(long)m * p.ldc + n + e] = f2bf(v);
            }
          }
        }
      }
    }
  }
}

bool gemm_w4_supported(const GemmArgs& a) {
  return a.conv == 0 && (!a.glu || a.N % 8 == 0) && a.batch <= 1 && a.in_scale == nullptr && a.bias2d == nullptr &&
         a.gate == nullptr && !a.rms && a.w_scale == nullptr && a.A2 == nullptr && a.K % 8 == 0 &&
         a.lda % 8 == 0 && a.ldw % 8 == 0 && (long)a.M * a.lda * 2 < 0x7fffffffL &&
         (long)a.N * a.ldw * 2 < 0x7fffffffL;
}

void launch_gemm_w4(const GemmArgs& a, hipStream_t s) {
  const int tiles = ((a.M + W4_BM - 1) / W4_BM) * ((a.N + W4_BN - 1) / W4_BN);
  const size_t lds = (size_t)2 * W4_STAGE * sizeof(bf16_t);
  if (a.glu) {
    switch (a.act) {
      case ACT_SILU: gemm_w4_kernel<ACT_SILU, true><<<tiles, 256, lds, s>>>(a); break;
      case ACT_GELU_TANH: gemm_w4_kernel<ACT_GELU_TANH, true><<<tiles, 256, lds, s>>>(a); break;
      default: gemm_w4_kernel<ACT_GELU, true><<<tiles, 256, lds, s>>>(a); break;
    }
    return;
  }
  switch (a.act) {
    case ACT_SILU: gemm_w4_kernel<ACT_SILU, false><<<tiles, 256, lds, s>>>(a); break;
    case ACT_GELU: gemm_w4_kernel<ACT_GELU, false><<<tiles, 256, lds, s>>>(a); break;
    case ACT_GELU_TANH: gemm_w4_kernel<ACT_GELU_TANH, false><<<tiles, 256, lds, s>>>(a); break;
    case ACT_QUICK_GELU: gemm_w4_kernel<ACT_QUICK_GELU, false><<<tiles, 256, lds, s>>>(a); break;
    case ACT_RELU: gemm_w4_kernel<ACT_RELU, false><<<tiles, 256, lds, s>>>(a); break;
    default: gemm_w4_kernel<ACT_NONE, false><<<tiles, 256, lds, s>>>(a); break;
  }
}

}  // namespace shai
