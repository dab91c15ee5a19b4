// bf16 GEMM for the low-K, 320-multiple-wide UNet projections (SD2.1 64x64 level: K = 320, N = 320 / 960 / 2560,
// M = 262144 at batch 32 with CFG): "W-stationary" persistent kernel, v6.
//
//   C[m, n] = act(alpha * rstd[m] (sum_k A[m, k] W[n, k] - mean[m] s[n]) + bias[n]) + res_alpha * R[m, n]
//   (the LayerNorm fold -- mean / rstd / s -- only with row_mr; GLU pairs (value, gate) columns)
//
// Why: with K = 320 a 256 x 320 output tile of the 8-phase kernel (gemm_8ph.hip) is 5 K-steps of MFMA work, and
// per tile the kernel pays a full operand-fetch latency (one K-step of lookahead) and a burst of 160 KB of output
// stores that the next tile's first `vmcnt` must drain: the round-5 lab measured the SD2.1 GEGLU 262144 x 2560 x 320
// at 575-600 TF/s (28 % of the MFMA time per tile) and proj 262144 x 320 x 320 (+res) at 3.9 TB/s.  Here:
//
// * The weights never move: each of the 4 waves (one per SIMD) keeps its 80 output columns x the whole K of W in
//   VGPRs (5 column blocks x K/32 k-steps of v_mfma_f32_16x16x32_bf16 A-operand fragments: 200 VGPRs at K = 320),
//   loaded once per workgroup.  A workgroup owns one 320-column slice of N for the whole launch.
// * Only A streams: BM x K row tiles (BM = 64, or 32 with a residual) land in LDS by LDS-DMA (`buffer_load ... lds`,
//   16 B per lane), NBUF = 3 tiles deep, so tile i + 2 is in flight while tile i computes (two tile-times of latency
//   cover, about 2.6 us at BM = 64).  The residual tile is staged the same way next to its A tile.
// * Stores overlap the next tile's MFMAs: tile i's epilogue stores are issued after tile i + 2's DMA, and the wait
//   for tile i + 1's operands is a counted `vmcnt` that leaves tile i's stores (and tile i + 2's DMA) in flight.
// * Every wave reads the full A tile (fragments by ds_read_b128, 64-wide K sub-tiles with the v4 bank swizzle):
//   50 B/clk/CU of LDS traffic at full MFMA rate, a fifth of the LDS bandwidth.
// * Workgroups on one XCD (blockIdx % 8) cover every N slice of the same M tiles at the same time, so each A tile
//   comes from HBM once per XCD and is re-read by the other N slices from that XCD's L2.
// * Each lane stores 8 consecutive columns per MFMA block pair (the W rows of a pair are permuted as in v4's wide
//   epilogue), 16-B stores; bias / LayerNorm column sums sit in LDS for the whole launch.
#include "gemm_epilogue.h"

#include <algorithm>

namespace shai {

typedef __bf16 wsbf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void ws_lds_void;

constexpr int WS_BN = 320, WS_WN = 80, WS_NB = 5;  // N slice per workgroup, columns per wave, 16-col blocks per wave
constexpr uint32_t WS_OOB = 0x80000000u;

template <int BM, int KT, bool RES, bool LNF, bool LNO = false>
struct WsT {
  static constexpr int RB = BM / 16;             // 16-row MFMA blocks per tile
  static constexpr int KS = 2 * KT;              // 32-deep k-steps
  static constexpr int A_BYTES = KT * BM * 128;  // K sub-tiles of [BM][64] bf16
  static constexpr int R_BYTES = RES ? BM * WS_BN * 2 : 0;
  static constexpr int MR_BYTES = LNF ? 1024 : 0;  // (mean, rstd) of the tile's rows, one 1 KB DMA instruction
  static constexpr int NA = 3, NR = 4;             // A ring (tile i + 2 in flight) / residual + row-moment ring
  static constexpr int RSLOT = R_BYTES + MR_BYTES;  // (tile i - 1's epilogue still reads its slot during tile i)
  static constexpr int COLS = LNF ? WS_BN * 4 : 0;  // LayerNorm column sums of the slice (fp32)
  static constexpr int RED = LNO ? 2 * 4 * BM * 4 : 0;  // LayerNorm-out row reduction: [pass][wave][row] fp32
  static constexpr int LDS = NA * A_BYTES + NR * RSLOT + COLS + RED;
  static constexpr int A_DMA = KT * BM / 32;    // A DMA instructions per wave per tile (8 rows x 128 B each)
  static constexpr int R_DMA = R_BYTES / 4096;  // residual DMA instructions per wave (1 KB each)
  static constexpr int DMA = A_DMA + R_DMA + (LNF ? 1 : 0);
  static constexpr int NCH = 3 * RB;            // epilogue chunks per tile: (row block, column group)
  static constexpr int NST = NCH * (LNO ? 2 : 1);  // store instructions per wave per full tile (one per chunk)
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(R_BYTES % 4096 == 0, "residual tile must split evenly over the 4 waves");
  static_assert(DMA + 2 * NST < 63, "vmcnt range");
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ws_rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)min(bytes, 0x7fffffffL),
                                           0x00020000);
}

// W-operand row r (0..15) of the wave's column block j -> column within the wave's 80: blocks (0,1) and (2,3) are
// permuted pairs (lane quad fq of the pair owns columns 32 q + 8 fq .. + 7), block 4 is the identity.
__device__ __forceinline__ int ws_wcol(int j, int r) {
  if (j < 4) return (j >> 1) * 32 + (r >> 2) * 8 + (j & 1) * 4 + (r & 3);
  return 64 + r;
}

// the residual tile's LDS image: row-major [BM][320] bf16 with 16-B chunks swizzled inside aligned groups of 8
__device__ __forceinline__ int ws_rchunk(int row, int ch) { return ch ^ (row & 7); }

typedef float wsf2 __attribute__((ext_vector_type(2)));
typedef __bf16 wsbf2 __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 pair (one v_cvt_pk_bf16_f32, round to nearest even)
__device__ __forceinline__ uint32_t ws_pk(float a, float b) {
  const wsf2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, wsbf2));
}

// LayerNorm of the output as a second output (LNO builds, N = 320: the whole row is in one workgroup):
// C2 = (y - mean(y)) rstd(y) gamma + beta over the stored (bf16) y -- the next LayerNorm computed in the producer's
// epilogue, two-pass (exact) moments from the registers.
struct WsLnOut {
  bf16_t* C2;
  const bf16_t* gamma;
  const bf16_t* beta;
  float eps;
};

// ABL (lab ablation builds only, 0 in production): bit 0 = no stores, bit 1 = no MFMA, bit 2 = no DMA after the prologue
template <int BM, int KT, int ACT, bool GLU, bool RES, bool LNF, bool LNO = false, int ABL = 0>
__global__ void __launch_bounds__(256, 1) gemm_ws_kernel(const GemmArgs p, int slots_per_xcd, int tiles_n,
                                                          const WsLnOut lo) {
  using T = WsT<BM, KT, RES, LNF, LNO>;
  constexpr int RB = T::RB, KS = T::KS;
  extern __shared__ __attribute__((aligned(16))) char ws_smem[];
  char* aring = ws_smem;                       // NA x A tile
  char* rring = ws_smem + T::NA * T::A_BYTES;  // NR x (residual tile | row moments)
  float* s_cols = reinterpret_cast<float*>(rring + T::NR * T::RSLOT);  // LayerNorm column sums
  float* s_red = reinterpret_cast<float*>(rring + T::NR * T::RSLOT + T::COLS);  // LNO row reduction

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;

  // ---- workgroup -> (N slice, M slot): blocks b and b + 8 share an XCD; the tiles_n workgroups of one XCD slot
  // cover every N slice of the same M tiles
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int nt = loc % tiles_n, sx = loc / tiles_n;
  if (sx >= slots_per_xcd) return;  // uniform: idle workgroup (32 % tiles_n leftovers)
  const int S = 8 * slots_per_xcd;   // M-tile stride of one workgroup
  const int slot = xcd + 8 * sx;
  const int n0 = nt * WS_BN;
  const int tiles_m = (p.M + BM - 1) / BM;

  // ---- W fragments: wave wid owns columns n0 + 80 wid .. + 79; lane (fr, fq) holds W[col(j, fr)][32 s + 8 fq ..].
  // They live in AGPRs (200 of them at K = 320, loaded straight into the accumulator file) and feed the MFMA's
  // A operand from there; the VGPRs hold two accumulator sets (this tile's and the previous tile's, whose epilogue
  // runs between this tile's MFMAs) and the X fragments.
  wsbf16x8 wf[WS_NB][KS];
#pragma unroll
  for (int j = 0; j < WS_NB; ++j) {
    const bf16_t* wrow = p.W + (long)(n0 + wid * WS_WN + ws_wcol(j, fr)) * p.ldw + 8 * fq;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const wsbf16x8 t = *reinterpret_cast<const wsbf16x8*>(wrow + 32 * s);
      asm volatile("; w -> agpr" : "=a"(wf[j][s]) : "0"(t));
    }
  }
  // the lane's 20 columns are fixed for the whole launch: the bias stays in registers (the LayerNorm column sums in
  // LDS).  Column group q: q < 2 -> 8 columns cw + 32 q + 8 fq .., q = 2 -> 4 columns cw + 64 + 4 fq ..
  const int cw = wid * WS_WN;
  float bq[3][8];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int c = n0 + (q < 2 ? cw + 32 * q + 8 * fq : cw + 64 + 4 * fq);
#pragma unroll
    for (int e = 0; e < 8; ++e) bq[q][e] = ((q < 2 || e < 4) && p.bias) ? bf2f(p.bias[c + e]) : 0.f;
  }
  if constexpr (LNF) {
    for (int c = tid; c < WS_BN; c += 256) s_cols[c] = p.col_s[n0 + c];  // read after the first tile's barrier
  }
  float gq[3][8], beq[3][8];  // LNO: the output LayerNorm's gain / shift of the lane's columns
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int c = n0 + (q < 2 ? cw + 32 * q + 8 * fq : cw + 64 + 4 * fq);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool v = LNO && (q < 2 || e < 4);
      gq[q][e] = v ? (lo.gamma ? bf2f(lo.gamma[c + e]) : 1.f) : 0.f;
      beq[q][e] = v ? (lo.beta ? bf2f(lo.beta[c + e]) : 0.f) : 0.f;
    }
  }

  // ---- DMA geometry
  const __amdgpu_buffer_rsrc_t rA = ws_rsrc(p.A, (long)p.M * p.lda * 2);
  const int lrow = lane >> 3, lpos = lane & 7;
  // A: instruction (t, h) stages rows 8 (wid * (BM / 32) + h) + lrow of K sub-tile t; source chunk swizzled
  constexpr int AH = BM / 32;  // 8-row groups per wave per K sub-tile
  uint32_t aoff[AH];
  int arow[AH];
#pragma unroll
  for (int h = 0; h < AH; ++h) {
    arow[h] = 8 * (wid * AH + h) + lrow;  // LDS row (0..BM-1)
    aoff[h] = (uint32_t)(((long)arow[h] * p.lda + (lpos ^ ((arow[h] >> 1) & 7)) * 8) * 2);
  }
  __amdgpu_buffer_rsrc_t rR;
  uint32_t roff[T::R_DMA > 0 ? T::R_DMA : 1];
  int rrow[T::R_DMA > 0 ? T::R_DMA : 1];
  if constexpr (RES) {
    rR = ws_rsrc(p.residual, (long)p.M * p.ldr * 2);
    // residual instruction q of this wave covers image bytes [1024 (wid * R_DMA + q), + 1024): lane -> (row, chunk)
#pragma unroll
    for (int q = 0; q < T::R_DMA; ++q) {
      const int byte = 1024 * (wid * T::R_DMA + q) + 16 * lane;
      const int row = byte / (WS_BN * 2), pos = (byte - row * WS_BN * 2) >> 4;
      const int ch = ws_rchunk(row, pos);  // the source chunk stored at image position pos
      rrow[q] = row;
      roff[q] = (uint32_t)(((long)row * p.ldr + n0 + 8 * ch) * 2);
    }
  }
  __amdgpu_buffer_rsrc_t rMR;
  if constexpr (LNF) rMR = ws_rsrc(p.row_mr, (long)p.M * 8);

  // issue every DMA instruction of this workgroup's i-th tile (A into ring slot i % NA, residual / row moments into
  // slot i % NR).  A tile past the end reads zeros: the instruction count per wave stays constant, so the counted
  // waits below hold.
  auto stage = [&](int i) {
    const int mt = slot + S * i;
    char* st = aring + (i % T::NA) * T::A_BYTES;
    char* rs = rring + (i % T::NR) * T::RSLOT;
    const int m0 = mt * BM;
    const int rows = mt < tiles_m ? p.M - m0 : 0;  // valid rows of the tile (may exceed BM)
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int h = 0; h < AH; ++h) {
        const uint32_t off = arow[h] < rows ? (uint32_t)m0 * (uint32_t)(p.lda * 2) + aoff[h] + 128u * t : WS_OOB;
        SHAI_DASSERT_DMA(off, (long)p.M * p.lda * 2, WS_OOB);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (ws_lds_void*)(st + t * BM * 128 + 8 * (wid * AH + h) * 128), 16,
                                                 off, 0, 0, 0);
      }
    if constexpr (RES) {
#pragma unroll
      for (int q = 0; q < T::R_DMA; ++q) {
        const uint32_t off = rrow[q] < rows ? (uint32_t)m0 * (uint32_t)(p.ldr * 2) + roff[q] : WS_OOB;
        SHAI_DASSERT_DMA(off, (long)p.M * p.ldr * 2, WS_OOB);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rR, (ws_lds_void*)(rs + 1024 * (wid * T::R_DMA + q)), 16, off, 0, 0,
                                                 0);
      }
    }
    if constexpr (LNF) {  // BM rows x 8 B: lane l brings rows 2l, 2l + 1; every wave issues the same bytes
      const uint32_t off = (2 * lane < BM && 2 * lane < rows) ? (uint32_t)(m0 + 2 * lane) * 8u : WS_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rMR, (ws_lds_void*)(rs + T::R_BYTES), 16, off, 0, 0, 0);
    }
  };

  // X-fragment LDS byte offset of row block rb, k-step s (K sub-tile s / 2, chunk 4 (s & 1) + fq, swizzled)
  auto xaddr = [&](int rb, int s) {
    const int row = 16 * rb + fr;
    return (s >> 1) * BM * 128 + row * 128 + (((4 * (s & 1) + fq) ^ ((row >> 1) & 7)) << 4);
  };

  // ---- epilogue chunk c = (row block rb, column group q) of the i-th tile from its accumulators: lane row
  // m0 + 16 rb + fr; one store instruction per chunk (16 B, or 8 B for the 4-column group; GLU halves both)
  // the chunk's LayerNorm constants, loaded ahead of its VALU work (a step earlier in the interleaved build)
  struct LnPre {
    float mean, rstd, sc[8];
  };
  auto epi_pre = [&](int c, int i) {
    LnPre l{0.f, 1.f, {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}};
    if constexpr (LNF) {
      const int rb = c / 3, q = c - 3 * rb;
      const char* rs = rring + (i % T::NR) * T::RSLOT;
      const int c0 = q < 2 ? cw + 32 * q + 8 * fq : cw + 64 + 4 * fq;
      const float2 mr = *reinterpret_cast<const float2*>(rs + T::R_BYTES + (16 * rb + fr) * 8);
      const float4_ s0 = *reinterpret_cast<const float4_*>(s_cols + c0);
      const float4_ s1 = q < 2 ? *reinterpret_cast<const float4_*>(s_cols + c0 + 4) : float4_{0.f, 0.f, 0.f, 0.f};
      l.mean = mr.x;
      l.rstd = mr.y;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        l.sc[e] = s0[e];
        l.sc[4 + e] = s1[e];
      }
    }
    return l;
  };
  auto epi_chunk = [&](const float4_ (&acc)[RB][WS_NB], int c, int i, const LnPre& ln) {
    const int rb = c / 3, q = c - 3 * rb;
    const int m0 = (slot + S * i) * BM;
    const char* rs = rring + (i % T::NR) * T::RSLOT;
    const int row = 16 * rb + fr;
    const long m = (long)m0 + row;
    const int nv = q < 2 ? 8 : 4;
    const int c0 = q < 2 ? cw + 32 * q + 8 * fq : cw + 64 + 4 * fq;  // first column within the slice
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = acc[rb][q < 2 ? 2 * q : 4][e];
      v[4 + e] = q < 2 ? acc[rb][2 * q + 1][e] : 0.f;
    }
    if constexpr (LNF) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ln.rstd * fmaf(-ln.mean, ln.sc[e], v[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fmaf(v[e], p.alpha, bq[q][e]);
    const bool ok = m < p.M && !(ABL & 1);
    if constexpr ((ABL & 1) != 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(v[e]));
    }
    if constexpr (GLU) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = v[2 * e] * apply_act<ACT>(v[2 * e + 1]);
      bf16_t* dst = p.C + m * p.ldc + ((n0 + c0) >> 1);
      if (ok) {
        if (nv == 8) {
          uint2_ w;
          w[0] = ws_pk(o[0], o[1]);
          w[1] = ws_pk(o[2], o[3]);
          *reinterpret_cast<uint2_*>(dst) = w;
        } else {
          *reinterpret_cast<uint32_t*>(dst) = ws_pk(o[0], o[1]);
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = apply_act<ACT>(v[e]);
      if constexpr (RES) {
        const char* rimg = rs + row * (WS_BN * 2);
        const int ch = c0 >> 3;
        float r8[8];
        if (nv == 8) {
          unpack8(*reinterpret_cast<const uint4_*>(rimg + (ws_rchunk(row, ch) << 4)), r8);
        } else {
          const uint2_ rr = *reinterpret_cast<const uint2_*>(rimg + (ws_rchunk(row, ch) << 4) + ((c0 & 4) ? 8 : 0));
          r8[0] = bf2f(rr[0] & 0xffff); r8[1] = bf2f(rr[0] >> 16);
          r8[2] = bf2f(rr[1] & 0xffff); r8[3] = bf2f(rr[1] >> 16);
          r8[4] = r8[5] = r8[6] = r8[7] = 0.f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaf(r8[e], p.res_alpha, v[e]);
      }
      bf16_t* dst = p.C + m * p.ldc + n0 + c0;
      if (ok) {
        if (nv == 8) {
          uint4_ w;
          w[0] = ws_pk(v[0], v[1]);
          w[1] = ws_pk(v[2], v[3]);
          w[2] = ws_pk(v[4], v[5]);
          w[3] = ws_pk(v[6], v[7]);
          *reinterpret_cast<uint4_*>(dst) = w;
        } else {
          uint2_ w;
          w[0] = ws_pk(v[0], v[1]);
          w[1] = ws_pk(v[2], v[3]);
          *reinterpret_cast<uint2_*>(dst) = w;
        }
      }
    }
  };

  // ---- GLU epilogue unit rb of the i-th tile (BM = 64: RB = 4 units): the row block's three column groups, stored
  // 16 B per lane.  Column groups 0 and 1 give each lane 4 + 4 outputs that are not adjacent; one v_permlane16_swap
  // per dword pairs lane quads (0, 1) and (2, 3) so each lane holds 8 consecutive outputs of one group (quad fq: group
  // fq & 1, outputs 8 (fq >> 1) ..).  Group 2 gives each lane one dword (2 outputs) per row block: they are parked in
  // d2[rb] and, after the last unit, a 4 x 4 transpose across the lane quads (v_permlane32_swap, then 16) leaves lane
  // quad fq with row block fq's 8 outputs.  RB + 1 store instructions per tile instead of 3 RB of 8 / 4 bytes: the
  // GEGLU epilogue was store-issue bound.
  auto epi_glu_unit = [&](const float4_ (&acc)[RB][WS_NB], int rb, int i, uint32_t (&d2)[RB]) {
    const int m0 = (slot + S * i) * BM;
    const long m = (long)m0 + 16 * rb + fr;
    uint32_t w[3][2];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const LnPre ln = epi_pre(3 * rb + q, i);
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[rb][q < 2 ? 2 * q : 4][e];
        v[4 + e] = q < 2 ? acc[rb][2 * q + 1][e] : 0.f;
      }
      if constexpr (LNF) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ln.rstd * fmaf(-ln.mean, ln.sc[e], v[e]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaf(v[e], p.alpha, bq[q][e]);
      if constexpr ((ABL & 1) != 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(v[e]));
      }
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = v[2 * e] * apply_act<ACT>(v[2 * e + 1]);
      w[q][0] = ws_pk(o[0], o[1]);
      w[q][1] = ws_pk(o[2], o[3]);
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const auto r = __builtin_amdgcn_permlane16_swap(w[0][e], w[1][e], false, false);
      w[0][e] = r[0];
      w[1][e] = r[1];
    }
    const int ob = (n0 + cw) >> 1;  // the wave's first output column
    if (m < p.M && !(ABL & 1))
      *reinterpret_cast<uint4_*>(p.C + m * p.ldc + ob + 16 * (fq & 1) + 8 * (fq >> 1)) =
          uint4_{w[0][0], w[0][1], w[1][0], w[1][1]};
    d2[rb] = w[2][0];
    if (rb == RB - 1) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const auto r = __builtin_amdgcn_permlane32_swap(d2[e], d2[2 + e], false, false);
        d2[e] = r[0];
        d2[2 + e] = r[1];
      }
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const auto r = __builtin_amdgcn_permlane16_swap(d2[2 * e], d2[2 * e + 1], false, false);
        d2[2 * e] = r[0];
        d2[2 * e + 1] = r[1];
      }
      const long m2 = (long)m0 + 16 * fq + fr;
      if (m2 < p.M && !(ABL & 1))
        *reinterpret_cast<uint4_*>(p.C + m2 * p.ldc + ob + 32) = uint4_{d2[0], d2[1], d2[2], d2[3]};
    }
  };

  // ---- LNO epilogue of the i-th tile (residual builds, no activation): y = acc + bias + res_alpha R stored to C,
  // then the row moments of the stored bf16 y across the 4 waves (LDS, raw barriers: an LDS-DMA prefetch is in
  // flight) and C2 = LayerNorm(y) gamma + beta
  auto epi_lnout = [&](const float4_ (&acc)[RB][WS_NB], int i) {
    const int m0 = (slot + S * i) * BM;
    const char* rs = rring + (i % T::NR) * T::RSLOT;
    float vv[RB][3][8];
    float ps[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int row = 16 * rb + fr;
      const long m = (long)m0 + row;
      const bool ok = m < p.M;
      ps[rb] = 0.f;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int nv = q < 2 ? 8 : 4;
        const int c0 = q < 2 ? cw + 32 * q + 8 * fq : cw + 64 + 4 * fq;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[rb][q < 2 ? 2 * q : 4][e];
          v[4 + e] = q < 2 ? acc[rb][2 * q + 1][e] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaf(v[e], p.alpha, bq[q][e]);
        if constexpr (RES) {
          const char* rimg = rs + row * (WS_BN * 2);
          const int ch = c0 >> 3;
          float r8[8];
          if (nv == 8) {
            unpack8(*reinterpret_cast<const uint4_*>(rimg + (ws_rchunk(row, ch) << 4)), r8);
          } else {
            const uint2_ rr = *reinterpret_cast<const uint2_*>(rimg + (ws_rchunk(row, ch) << 4) + ((c0 & 4) ? 8 : 0));
            r8[0] = bf2f(rr[0] & 0xffff); r8[1] = bf2f(rr[0] >> 16);
            r8[2] = bf2f(rr[1] & 0xffff); r8[3] = bf2f(rr[1] >> 16);
            r8[4] = r8[5] = r8[6] = r8[7] = 0.f;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaf(r8[e], p.res_alpha, v[e]);
        }
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = ws_pk(v[2 * e], v[2 * e + 1]);
        // the moments are those of the stored (bf16) values: what the reference LayerNorm reads
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          vv[rb][q][2 * e] = __uint_as_float(w[e] << 16);
          vv[rb][q][2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (e < nv) ps[rb] += vv[rb][q][e];
        bf16_t* dst = p.C + m * p.ldc + n0 + c0;
        if (ok) {
          if (nv == 8) *reinterpret_cast<uint4_*>(dst) = uint4_{w[0], w[1], w[2], w[3]};
          else *reinterpret_cast<uint2_*>(dst) = uint2_{w[0], w[1]};
        }
      }
    }
    // pass 1: row sums -> mean; pass 2: sums of squared deviations -> rstd
    float mean[RB], rstd[RB];
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        float t = ps[rb];
        t += __shfl_xor(t, 16, 64);
        t += __shfl_xor(t, 32, 64);
        if (fq == 0) s_red[(pass * 4 + wid) * BM + 16 * rb + fr] = t;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const int row = 16 * rb + fr;
        const float tot = (s_red[(pass * 4 + 0) * BM + row] + s_red[(pass * 4 + 1) * BM + row]) +
                          (s_red[(pass * 4 + 2) * BM + row] + s_red[(pass * 4 + 3) * BM + row]);
        if (pass == 0) {
          mean[rb] = tot * (1.f / WS_BN);
          float d = 0.f;
#pragma unroll
          for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (q < 2 || e < 4) d = fmaf(vv[rb][q][e] - mean[rb], vv[rb][q][e] - mean[rb], d);
          ps[rb] = d;
        } else {
          rstd[rb] = rsqrtf(tot * (1.f / WS_BN) + lo.eps);
        }
      }
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const long m = (long)m0 + 16 * rb + fr;
      const bool ok = m < p.M;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int nv = q < 2 ? 8 : 4;
        const int c0 = q < 2 ? cw + 32 * q + 8 * fq : cw + 64 + 4 * fq;
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = fmaf((vv[rb][q][e] - mean[rb]) * rstd[rb], gq[q][e], beq[q][e]);
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = ws_pk(o[2 * e], o[2 * e + 1]);
        bf16_t* dst = lo.C2 + m * p.ldc + n0 + c0;
        if (ok) {
          if (nv == 8) *reinterpret_cast<uint4_*>(dst) = uint4_{w[0], w[1], w[2], w[3]};
          else *reinterpret_cast<uint2_*>(dst) = uint2_{w[0], w[1]};
        }
      }
    }
  };

  // ---- one tile: wait for its DMA, put tile i + 2's in flight, then 2 KT k-steps x RB x 5 MFMAs (X fragments read
  // one k-step ahead) with the previous tile's epilogue chunks spread between the MFMA groups, so its VALU work and
  // store issue overlap this tile's matrix pipe.  The MFMAs are inline asm: the weight operand must be read from the
  // AGPRs it lives in (the builtin would copy it into VGPRs first).  Hazards the compiler cannot see into the asm:
  // an accumulator is re-read as C 5 RB MFMAs after it was written; the previous tile's accumulators were finished a
  // whole tile (and a barrier) ago; the final epilogue waits behind s_nops.
  // IL (the GLU build, whose epilogue is VALU-heavy: GELU / SiLU per output pair): the previous tile's epilogue
  // chunks run between this tile's MFMA groups.  Otherwise (plain / bias / residual: a few VALU per output) each tile's
  // epilogue follows its own MFMAs, which measured faster there (round-5 lab: no second accumulator set to keep).
  constexpr bool IL = GLU;
  static_assert(!GLU || RB == 4, "the GLU epilogue's lane-quad transpose assumes 4 row blocks");
  constexpr int NU = GLU ? RB : T::NCH;        // epilogue units per tile
  constexpr int NST = GLU ? RB + 1 : T::NST;   // store instructions per wave per full tile
  auto tile = [&](float4_ (&acc)[RB][WS_NB], const float4_ (&prev)[RB][WS_NB], int i) {
    // outstanding after tile i's DMA: tile i + 1's DMA and the stores of tiles i - 2 and i - 1
    if constexpr (SHAI_DEBUG) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // debug: hazard-safe drain
    else if (i >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T::DMA + 2 * NST) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T::DMA) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the slots restaged next are done
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!(ABL & 4)) stage(i + 2);  // A slot of tile i - 1, residual slot of tile i - 2: every wave is past its reads
    __builtin_amdgcn_sched_barrier(0);
    const bool has_prev = i > 0;
    const char* sa = aring + (i % T::NA) * T::A_BYTES;
    // steps (rb, s) in row-block-major order: 5 MFMAs each (one per column block) on the X fragment of row block rb,
    // k-step s, read two steps ahead.  Row-block-major keeps a row block's accumulators dead until its first step, so
    // the previous tile's accumulators (consumed by the epilogue chunks in the first half of the steps) and this
    // tile's share registers: at most 1.5 accumulator sets are live.
    constexpr int NSTEP = RB * KS;
    uint32_t d2[RB];  // GLU: group-2 dwords of the previous tile's row blocks, stored after its last unit
    wsbf16x8 xr[3];
    xr[0] = *reinterpret_cast<const wsbf16x8*>(sa + xaddr(0, 0));
    xr[1] = *reinterpret_cast<const wsbf16x8*>(sa + xaddr(1 / KS, 1 % KS));
#pragma unroll
    for (int st = 0; st < NSTEP; ++st) {
      const int rb = st / KS, s = st % KS;
      if (st + 2 < NSTEP) xr[(st + 2) % 3] = *reinterpret_cast<const wsbf16x8*>(sa + xaddr((st + 2) / KS, (st + 2) % KS));
      __builtin_amdgcn_sched_barrier(0);  // the read two steps ahead goes out before this step's MFMAs
      const wsbf16x8& xc = xr[st % 3];
#pragma unroll
      for (int j = 0; j < WS_NB; ++j) {
        if constexpr ((ABL & 2) != 0) {  // lab ablation: no MFMA (operands kept live)
          asm volatile("; nomfma" : "=v"(acc[rb][j]) : "a"(wf[j][s]), "v"(xc));
          continue;
        }
        if (s == 0)
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(acc[rb][j]) : "a"(wf[j][s]), "v"(xc));
        else
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[rb][j]) : "a"(wf[j][s]), "v"(xc));
      }
      if constexpr (SHAI_DEBUG) asm volatile("s_nop 7" ::: "memory");  // debug: wide hazard margin
      else asm volatile("s_nop 1" ::: "memory");  // WAR margin: a later read may land in this step's X registers
      // epilogue units of the previous tile, spread over the first half of the steps
      if constexpr (IL) {
#pragma unroll
        for (int c = 0; c < NU; ++c) {
          if (st == (c * (NSTEP / 2)) / NU) {
            __builtin_amdgcn_sched_barrier(0);
            if (has_prev) epi_glu_unit(prev, c, i - 1, d2);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    }
    if constexpr (!IL) {  // this tile's own epilogue right after its MFMAs
      asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");  // MFMA results -> VALU reads
      if constexpr (LNO) {
        epi_lnout(acc, i);
      } else {
#pragma unroll
        for (int c = 0; c < T::NCH; ++c) epi_chunk(acc, c, i, epi_pre(c, i));
      }
    }
  };

  const int i_end = slot < tiles_m ? (tiles_m - 1 - slot) / S + 1 : 0;  // tiles of this workgroup
  // prologue: tiles 0 and 1 of this workgroup in flight
  stage(0);
  stage(1);
  float4_ accA[RB][WS_NB], accB[RB][WS_NB];
  for (int i = 0; i < i_end; i += 2) {
    tile(accA, accB, i);
    if (i + 1 < i_end) tile(accB, accA, i + 1);
  }
  // the last tile's epilogue (its MFMA results: s_nops for the VALU reads)
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  if constexpr (IL) {
    if (i_end > 0) {
      const int il = i_end - 1;
      uint32_t d2[RB];
#pragma unroll
      for (int c = 0; c < NU; ++c) {
        if (il & 1) epi_glu_unit(accB, c, il, d2);
        else epi_glu_unit(accA, c, il, d2);
      }
    }
  }
  // every LDS-DMA of this workgroup (prefetches past the end included) lands before the LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------- host side
bool gemm_ws_supported(const GemmArgs& a) {
  if (a.conv || a.batch > 1 || a.A2 || a.in_scale || a.rms || a.w_scale || a.gate || a.bias2d) return false;
  if (a.K != 320 || a.N % WS_BN != 0 || a.M <= 0) return false;
  if (a.glu && a.residual) return false;
  if (a.lda % 8 || a.ldw % 8 || a.ldc % 8 || (a.residual && a.ldr % 8)) return false;
  const auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (!al(a.A) || !al(a.W) || !al(a.C) || (a.residual && !al(a.residual))) return false;
  if ((long)a.M * a.lda * 2 >= 0x7fffffffL || (a.residual && (long)a.M * a.ldr * 2 >= 0x7fffffffL)) return false;
  // exactly the variants launch_gemm_ws instantiates -- anything else would run as another activation (or drop
  // the folded LayerNorm) without an error:
  //   GLU:     SILU / GELU / GELU_TANH; the folded LayerNorm (row_mr) only with GELU
  //   non-GLU: NONE / SILU / GELU;      the folded LayerNorm only with NONE
  if (a.glu) {
    if (a.act != ACT_SILU && a.act != ACT_GELU && a.act != ACT_GELU_TANH) return false;
    if (a.row_mr && a.act != ACT_GELU) return false;
  } else {
    if (a.act != ACT_NONE && a.act != ACT_SILU && a.act != ACT_GELU) return false;
    if (a.row_mr && a.act != ACT_NONE) return false;
  }
  if (a.row_mr && a.col_s == nullptr) return false;
  return true;
}

static int ws_grid() {
  static int w = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 8)
      cus = 256;
    return cus & ~7;
  }();
  return w;
}

// lab-only ablation switch (tools/gemm_lab: stores / MFMA / DMA skipped to price each); 0 in production
static int ws_ablation = 0;
void gemm_ws_set_ablation(int a) { ws_ablation = a; }

template <int BM, int ACT, bool GLU, bool RES, bool LNF, bool LNO = false>
static void ws_go(const GemmArgs& a, hipStream_t s, const WsLnOut& lo = WsLnOut{nullptr, nullptr, nullptr, 0.f}) {
  using T = WsT<BM, 5, RES, LNF, LNO>;
  const int tiles_n = a.N / WS_BN;
  const int per_xcd = ws_grid() / 8;
  int spx = per_xcd / tiles_n;
  if (spx < 1) spx = 1;
  const int grid = 8 * std::max(per_xcd, tiles_n);
#ifdef SHAI_GEMM_LAB
  switch (ws_ablation) {
    case 1: gemm_ws_kernel<BM, 5, ACT, GLU, RES, LNF, LNO, 1><<<grid, 256, T::LDS, s>>>(a, spx, tiles_n, lo); return;
    case 2: gemm_ws_kernel<BM, 5, ACT, GLU, RES, LNF, LNO, 2><<<grid, 256, T::LDS, s>>>(a, spx, tiles_n, lo); return;
    case 3: gemm_ws_kernel<BM, 5, ACT, GLU, RES, LNF, LNO, 3><<<grid, 256, T::LDS, s>>>(a, spx, tiles_n, lo); return;
    case 4: gemm_ws_kernel<BM, 5, ACT, GLU, RES, LNF, LNO, 4><<<grid, 256, T::LDS, s>>>(a, spx, tiles_n, lo); return;
    default: break;
  }
#endif
  gemm_ws_kernel<BM, 5, ACT, GLU, RES, LNF, LNO><<<grid, 256, T::LDS, s>>>(a, spx, tiles_n, lo);
}

template <int ACT, bool GLU>
static void ws_res(const GemmArgs& a, hipStream_t s) {
  if (a.residual) ws_go<32, ACT, GLU, true, false>(a, s);
  else ws_go<64, ACT, GLU, false, false>(a, s);
}

void launch_gemm_ws(const GemmArgs& a, hipStream_t s) {
  if (a.glu) {
    if (a.act == ACT_SILU) ws_go<64, ACT_SILU, true, false, false>(a, s);
    else if (a.act == ACT_GELU_TANH) ws_go<64, ACT_GELU_TANH, true, false, false>(a, s);
    else if (a.row_mr) ws_go<64, ACT_GELU, true, false, true>(a, s);
    else ws_go<64, ACT_GELU, true, false, false>(a, s);
    return;
  }
  if (a.row_mr) {  // folded LayerNorm (SD2.1 QKV / Q): no activation
    if (a.residual) ws_go<32, ACT_NONE, false, true, true>(a, s);
    else ws_go<64, ACT_NONE, false, false, true>(a, s);
    return;
  }
  switch (a.act) {
    case ACT_SILU: ws_res<ACT_SILU, false>(a, s); break;
    case ACT_GELU: ws_res<ACT_GELU, false>(a, s); break;
    default: ws_res<ACT_NONE, false>(a, s); break;
  }
}

// y = x W^T + bias + res_alpha R into C and LayerNorm(y) gamma + beta into C2 (N = 320, residual, no activation).
bool gemm_ws_lnout_supported(const GemmArgs& a) {
  return gemm_ws_supported(a) && a.N == WS_BN && a.residual != nullptr && !a.glu && a.act == ACT_NONE &&
         a.row_mr == nullptr;
}

void launch_gemm_ws_lnout(const GemmArgs& a, bf16_t* C2, const bf16_t* gamma, const bf16_t* beta, float eps,
                          hipStream_t s) {
  ws_go<32, ACT_NONE, false, true, false, true>(a, s, WsLnOut{C2, gamma, beta, eps});
}

}  // namespace shai
