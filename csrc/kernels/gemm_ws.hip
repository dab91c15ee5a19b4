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

template <int BM, int KT, bool RES, bool LNF>
struct WsT {
  static constexpr int RB = BM / 16;            // 16-row MFMA blocks per tile
  static constexpr int KS = 2 * KT;             // 32-deep k-steps
  static constexpr int A_BYTES = KT * BM * 128;  // K sub-tiles of [BM][64] bf16
  static constexpr int R_BYTES = RES ? BM * WS_BN * 2 : 0;
  static constexpr int MR_BYTES = LNF ? 1024 : 0;  // (mean, rstd) of the tile's rows, one 1 KB DMA instruction
  static constexpr int STAGE = A_BYTES + R_BYTES + MR_BYTES;
  static constexpr int NBUF = 3;
  static constexpr int COL_BYTES = 2 * WS_BN * 4;  // bias, LayerNorm column sums (fp32)
  static constexpr int LDS = COL_BYTES + NBUF * STAGE;
  static constexpr int A_DMA = KT * BM / 32;    // A DMA instructions per wave per tile (8 rows x 128 B each)
  static constexpr int R_DMA = R_BYTES / 4096;  // residual DMA instructions per wave (1 KB each)
  static constexpr int DMA = A_DMA + R_DMA + (LNF ? 1 : 0);
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(R_BYTES % 4096 == 0, "residual tile must split evenly over the 4 waves");
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

template <int BM, int KT, int ACT, bool GLU, bool RES, bool LNF>
__global__ void __launch_bounds__(256, 1) gemm_ws_kernel(const GemmArgs p, int slots_per_xcd, int tiles_n) {
  using T = WsT<BM, KT, RES, LNF>;
  constexpr int RB = T::RB, KS = T::KS;
  extern __shared__ __attribute__((aligned(16))) char ws_smem[];
  float* s_bias = reinterpret_cast<float*>(ws_smem);
  float* s_cols = s_bias + WS_BN;
  char* stages = ws_smem + T::COL_BYTES;

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

  // ---- W fragments: wave wid owns columns n0 + 80 wid .. + 79; lane (fr, fq) holds W[col(j, fr)][32 s + 8 fq ..]
  wsbf16x8 wf[WS_NB][KS];
#pragma unroll
  for (int j = 0; j < WS_NB; ++j) {
    const bf16_t* wrow = p.W + (long)(n0 + wid * WS_WN + ws_wcol(j, fr)) * p.ldw + 8 * fq;
#pragma unroll
    for (int s = 0; s < KS; ++s) wf[j][s] = *reinterpret_cast<const wsbf16x8*>(wrow + 32 * s);
  }
  // per-column epilogue constants of this N slice (fp32 in LDS for the whole launch)
  for (int c = tid; c < WS_BN; c += 256) {
    s_bias[c] = p.bias ? bf2f(p.bias[n0 + c]) : 0.f;
    if constexpr (LNF) s_cols[c] = p.col_s[n0 + c];
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
  if constexpr (RES) {
    rR = ws_rsrc(p.residual, (long)p.M * p.ldr * 2);
    // residual instruction q of this wave covers image bytes [1024 (wid * R_DMA + q), + 1024): lane -> (row, chunk)
#pragma unroll
    for (int q = 0; q < T::R_DMA; ++q) {
      const int byte = 1024 * (wid * T::R_DMA + q) + 16 * lane;
      const int row = byte / (WS_BN * 2), pos = (byte - row * WS_BN * 2) >> 4;
      const int ch = ws_rchunk(row, pos);  // the source chunk stored at image position pos
      roff[q] = (uint32_t)(((long)row * p.ldr + n0 + 8 * ch) * 2);
    }
  }
  __amdgpu_buffer_rsrc_t rMR;
  if constexpr (LNF) rMR = ws_rsrc(p.row_mr, (long)p.M * 8);

  // issue every DMA instruction of M tile `mt` into buffer `buf` (a tile past the end reads zeros: the instruction
  // count per wave stays constant, so the counted waits below hold)
  auto stage = [&](int buf, int mt) {
    char* st = stages + buf * T::STAGE;
    const long m0 = (long)mt * BM;
    const bool live = mt < tiles_m;
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int h = 0; h < AH; ++h) {
        const bool ok = live && m0 + arow[h] < p.M;
        const uint32_t off = ok ? (uint32_t)(m0 * p.lda * 2) + aoff[h] + 128u * t : WS_OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (ws_lds_void*)(st + t * BM * 128 + 8 * (wid * AH + h) * 128), 16,
                                                 off, 0, 0, 0);
      }
    if constexpr (RES) {
#pragma unroll
      for (int q = 0; q < T::R_DMA; ++q) {
        const int row = (1024 * (wid * T::R_DMA + q) + 16 * lane) / (WS_BN * 2);
        const bool ok = live && m0 + row < p.M;
        const uint32_t off = ok ? (uint32_t)(m0 * p.ldr * 2) + roff[q] : WS_OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rR, (ws_lds_void*)(st + T::A_BYTES + 1024 * (wid * T::R_DMA + q)), 16,
                                                 off, 0, 0, 0);
      }
    }
    if constexpr (LNF) {  // BM rows x 8 B: lane l brings rows 2l, 2l + 1; every wave issues the same bytes
      const bool ok = live && lane * 2 < BM && m0 + 2 * lane < p.M;
      const uint32_t off = ok ? (uint32_t)((m0 + 2 * lane) * 8) : WS_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rMR, (ws_lds_void*)(st + T::A_BYTES + T::R_BYTES), 16, off, 0, 0, 0);
    }
  };

  const int i_end = slot < tiles_m ? (tiles_m - 1 - slot) / S + 1 : 0;  // tiles of this workgroup
  // prologue: tiles 0 and 1 of this workgroup in flight
  stage(0, slot);
  stage(1, slot + S);

  // X-fragment LDS byte offset of row block rb, k-step s (K sub-tile s / 2, chunk 4 (s & 1) + fq, swizzled)
  auto xaddr = [&](int rb, int s) {
    const int row = 16 * rb + fr;
    return (s >> 1) * BM * 128 + row * 128 + (((4 * (s & 1) + fq) ^ ((row >> 1) & 7)) << 4);
  };

  float4_ acc[RB][WS_NB];
  bool drained = true;  // the previous epilogue issued its full, fixed store count (counted wait is exact)
  for (int i = 0; i < i_end; ++i) {
    const int buf = i % 3;
    const int mt = slot + S * i;
    const int m0 = mt * BM;
    // ---- wait for this tile's DMA; tile i - 1's stores and tile i + 1's DMA may stay in flight
    if (i == 0 || !drained) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T::DMA) : "memory");  // prologue: only tile 1's DMA after it
      if (!drained) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T::DMA + 3 * RB) : "memory");  // + tile i - 1's 3 RB stores
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the buffer restaged next are done
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    stage((i + 2) % 3, mt + 2 * S);  // into the buffer tile i - 1 used: every wave is past its reads (barrier)
    __builtin_amdgcn_sched_barrier(0);

    // ---- MFMA: 2 KT k-steps x RB x 5 blocks, X fragments read one k-step ahead
    const char* sa = stages + buf * T::STAGE;
    wsbf16x8 x0[RB], x1[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) x0[rb] = *reinterpret_cast<const wsbf16x8*>(sa + xaddr(rb, 0));
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      wsbf16x8* xc = (s & 1) ? x1 : x0;
      wsbf16x8* xn = (s & 1) ? x0 : x1;
      if (s + 1 < KS) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) xn[rb] = *reinterpret_cast<const wsbf16x8*>(sa + xaddr(rb, s + 1));
      }
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int j = 0; j < WS_NB; ++j)
          acc[rb][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][s], xc[rb], s == 0 ? float4_{0.f, 0.f, 0.f, 0.f}
                                                                                        : acc[rb][j],
                                                               0, 0, 0);
    }

    // ---- epilogue: lane row m0 + 16 rb + fr; columns (wave) 32 q + 8 fq .. + 7 for pairs q = 0, 1, 64 + 4 fq .. + 3
    const bool full = m0 + BM <= p.M;
    drained = full;
    const int cw = wid * WS_WN;  // wave's first column within the slice
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int row = 16 * rb + fr;
      const long m = (long)m0 + row;
      float mean = 0.f, rstd = 1.f;
      if constexpr (LNF) {
        const float2 mr = *reinterpret_cast<const float2*>(sa + T::A_BYTES + T::R_BYTES + row * 8);
        mean = mr.x;
        rstd = mr.y;
      }
      bf16_t* crow = p.C + m * p.ldc;
      const bool ok = m < p.M;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int nv = q < 2 ? 8 : 4;      // columns this lane owns in the group
        const int c = q < 2 ? cw + 32 * q + 8 * fq : cw + 64 + 4 * fq;
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[rb][q < 2 ? 2 * q : 4][e];
          if (q < 2) v[4 + e] = acc[rb][2 * q + 1][e];
        }
        float bb[8], cs[8];
        {
          const float4_ b0 = *reinterpret_cast<const float4_*>(s_bias + c);
          bb[0] = b0[0]; bb[1] = b0[1]; bb[2] = b0[2]; bb[3] = b0[3];
          if (q < 2) {
            const float4_ b1 = *reinterpret_cast<const float4_*>(s_bias + c + 4);
            bb[4] = b1[0]; bb[5] = b1[1]; bb[6] = b1[2]; bb[7] = b1[3];
          }
          if constexpr (LNF) {
            const float4_ c0 = *reinterpret_cast<const float4_*>(s_cols + c);
            cs[0] = c0[0]; cs[1] = c0[1]; cs[2] = c0[2]; cs[3] = c0[3];
            if (q < 2) {
              const float4_ c1 = *reinterpret_cast<const float4_*>(s_cols + c + 4);
              cs[4] = c1[0]; cs[5] = c1[1]; cs[6] = c1[2]; cs[7] = c1[3];
            }
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (e >= nv) break;
          float x = v[e];
          if constexpr (LNF) x = rstd * fmaf(-mean, cs[e], x);
          v[e] = fmaf(x, p.alpha, bb[e]);
        }
        if constexpr (GLU) {
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (2 * e >= nv) break;
            o[e] = v[2 * e] * apply_act<ACT>(v[2 * e + 1]);
          }
          bf16_t* dst = crow + ((n0 + c) >> 1);
          if (ok) {
            if (q < 2) {
              uint2_ w;
              w[0] = pack2(o[0], o[1]);
              w[1] = pack2(o[2], o[3]);
              *reinterpret_cast<uint2_*>(dst) = w;
            } else {
              *reinterpret_cast<uint32_t*>(dst) = pack2(o[0], o[1]);
            }
          }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            if (e >= nv) break;
            v[e] = apply_act<ACT>(v[e]);
          }
          if constexpr (RES) {
            const char* rimg = sa + T::A_BYTES + row * (WS_BN * 2);
            float r8[8];
            if (q < 2) {
              const int ch = c >> 3;
              unpack8(*reinterpret_cast<const uint4_*>(rimg + (ws_rchunk(row, ch) << 4)), r8);
            } else {
              const int ch = c >> 3;
              const uint2_ rr = *reinterpret_cast<const uint2_*>(rimg + (ws_rchunk(row, ch) << 4) + ((c & 4) ? 8 : 0));
              r8[0] = bf2f(rr[0] & 0xffff); r8[1] = bf2f(rr[0] >> 16);
              r8[2] = bf2f(rr[1] & 0xffff); r8[3] = bf2f(rr[1] >> 16);
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              if (e >= nv) break;
              v[e] = fmaf(r8[e], p.res_alpha, v[e]);
            }
          }
          bf16_t* dst = crow + n0 + c;
          if (ok) {
            if (q < 2) {
              *reinterpret_cast<uint4_*>(dst) = pack8(v);
            } else {
              uint2_ w;
              w[0] = pack2(v[0], v[1]);
              w[1] = pack2(v[2], v[3]);
              *reinterpret_cast<uint2_*>(dst) = w;
            }
          }
        }
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

template <int BM, int ACT, bool GLU, bool RES, bool LNF>
static void ws_go(const GemmArgs& a, hipStream_t s) {
  using T = WsT<BM, 5, RES, LNF>;
  const int tiles_n = a.N / WS_BN;
  const int per_xcd = ws_grid() / 8;
  int spx = per_xcd / tiles_n;
  if (spx < 1) spx = 1;
  const int grid = 8 * std::max(per_xcd, tiles_n);
  gemm_ws_kernel<BM, 5, ACT, GLU, RES, LNF><<<grid, 256, T::LDS, s>>>(a, spx, tiles_n);
}

template <int ACT, bool GLU>
static void ws_res_ln(const GemmArgs& a, hipStream_t s) {
  if (a.residual) {
    if (a.row_mr) ws_go<32, ACT, GLU, true, true>(a, s);
    else ws_go<32, ACT, GLU, true, false>(a, s);
  } else {
    if (a.row_mr) ws_go<64, ACT, GLU, false, true>(a, s);
    else ws_go<64, ACT, GLU, false, false>(a, s);
  }
}

void launch_gemm_ws(const GemmArgs& a, hipStream_t s) {
  if (a.glu) {
    if (a.act == ACT_SILU) ws_go<64, ACT_SILU, true, false, false>(a, s);
    else if (a.act == ACT_GELU_TANH) ws_go<64, ACT_GELU_TANH, true, false, false>(a, s);
    else if (a.row_mr) ws_go<64, ACT_GELU, true, false, true>(a, s);
    else ws_go<64, ACT_GELU, true, false, false>(a, s);
    return;
  }
  switch (a.act) {
    case ACT_SILU: ws_res_ln<ACT_SILU, false>(a, s); break;
    case ACT_GELU: ws_res_ln<ACT_GELU, false>(a, s); break;
    default: ws_res_ln<ACT_NONE, false>(a, s); break;
  }
}

}  // namespace shai
