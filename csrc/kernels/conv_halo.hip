// Halo-tiled implicit-GEMM 3x3 convolution (stride 1, pad 1, NHWC) with the GroupNorm + SiLU of its input applied
// ONCE per staged element, in LDS.
//
//   C[m, n] = sum_{kh, kw, c} silu(x[img, y + kh - 1, x + kw - 1, c] * scale[img, c] + shift[img, c]) W[n, kh, kw, c]
//             + bias[n] + bias2d[img, n] + res_alpha R[m, n]          (zero padding applied AFTER the norm)
//
// Why (round-5 verdict, SURVEY 2.4 / 2.9 "NHWC implicit-GEMM conv + fused GroupNorm-SiLU"): the tile GEMM kernels
// stage A by LDS-DMA, which cannot transform data in flight, so every GroupNorm + SiLU before a 3x3 conv was its own
// full read + write pass over the activation (gn_apply: ~7 % of the SD2.1 UNet step), and normalising inside a
// 9-tap gather instead repeats the transform 9 x per N-tile (VALU-bound, measured 5 x slower).  Here a workgroup
// owns TR whole output rows of one image (256 pixels: 4 x 64, 8 x 32 or 16 x 16) and walks the input channels in
// chunks of 64:
//
// * Halo: the (TR + 2) x (OW + 2) input pixels of the chunk (zero padding rows / columns included) land in LDS by
//   LDS-DMA, 16-B slot s of halo pixel P holding channels 8 (s ^ (P & 7)) .. + 7 (the XOR swizzle is on the source
//   address: the DMA image stays lane-linear).  Each lane then normalises exactly the 16-B slots its own DMA wrote
//   (ds_read -> fma + SiLU -> ds_write, ordered by that wave's vmcnt alone: no cross-wave hand-off) -- once per
//   element per N-tile; padding pixels keep the DMA's zero fill.  The per-(image, channel) scale / shift come from
//   the producer's GroupNorm partials (groupnorm_stats_from_partials) by one more LDS-DMA per chunk.
// * Taps: the 9 filter taps of a chunk are 9 K-tiles of 64 that read the SAME halo image at a constant pixel shift
//   (kh (OW + 2) + kw): the A fragments of a 16-pixel MFMA block are 16 consecutive halo pixels, conflict-free for
//   ds_read_b128 at every shift thanks to the swizzle (checked exhaustively on the host model).
// * W: per K-tile a [BN][64] slice of W[n, kh, kw, c] by LDS-DMA into a 2-stage ring (row-pair swizzle as the
//   four-wave kernel); the halo is double-buffered, so chunk c + 1's DMA + normalisation run under chunk c's taps.
// * Pipeline per K-tile (one barrier, as gemm_w4.hip): (a) k-step 0 MFMAs || k-step 1 fragment reads; (b) lgkmcnt(0)
//   + vmcnt(0) + s_barrier; (c) W DMA of tile t + 2 (and, at a chunk's first tap, the next chunk's halo + scale /
//   shift), tile t + 1's k-step 0 reads, k-step 1 MFMAs, and one slot group of the next chunk's normalisation.
// * Epilogue: bias / per-image bias2d (time embedding) / residual, and the GroupNorm column partials of the stored
//   output for the NEXT norm (GemmArgs::col_part, [M / 128, N, 2] (sum, sum of squares)).
//
// Also runs without a norm (MODE 0) and over a nearest-2x upsampled input (UPS: the halo DMA reads source pixel
// (y / 2, x / 2)), and with a two-source channel concat (A2 from channel Cin1, 64-aligned).
#include "gemm_epilogue.h"

#include <type_traits>
#include <utility>

namespace shai {

typedef __bf16 hcbf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void hc_lds_void;

constexpr int HC_BM = 256;           // output pixels per tile
constexpr int HC_BK = 64;            // channels per chunk = K per tile
constexpr int HC_HPIX_MAX = 448;     // halo pixels per buffer (>= 6 x 66 = 396, the largest supported halo)
constexpr uint32_t HC_OOB = 0x80000000u;

struct HaloGeo {
  int TR, HC, HPIX;   // output rows per tile, halo row length (OW + 2), halo pixels (TR + 2) (OW + 2)
  int lg_ow;          // log2 OW
  int tiles_m, tiles_n, nchunks;
};

template <int WAVES, int BNB>
struct HcT {
  static constexpr int WN_WAVES = WAVES / 4;             // waves: 4 (rows) x WN_WAVES (columns)
  static constexpr int BMB = 4;                          // 16-pixel blocks per wave (64 pixels)
  static constexpr int WN = 16 * BNB;                    // columns per wave
  static constexpr int BN = WN * WN_WAVES;
  static constexpr int HALO_ELEMS = HC_HPIX_MAX * HC_BK;
  static constexpr int W_ELEMS = BN * HC_BK;
  static constexpr int HJ = HC_HPIX_MAX / 8 / WAVES;     // halo DMA instructions (8 pixels each) per wave per chunk
  static constexpr int WJ = (BN / 8 + WAVES - 1) / WAVES;  // W DMA instructions per wave per K-tile (upper bound)
  static constexpr int SS_FLOATS = 256;                  // scale[64] | shift[64] | DMA zero fill
  static constexpr int LDS = (2 * HALO_ELEMS + 2 * W_ELEMS) * 2 + 2 * SS_FLOATS * 4;
  static_assert(HJ * 8 * WAVES == HC_HPIX_MAX, "halo DMA geometry");
  static_assert(LDS <= 163840, "LDS budget");
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t hc_rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)min(bytes, 0x7fffffffL),
                                           0x00020000);
}

// MODE: 0 = the input as is, 2 = GroupNorm + SiLU in LDS.  UPS: nearest-2x upsampled input (MODE 0 only).
// SGB (lab A/B): the normalisation hand-interleaved with the step's MFMAs, one 3-op phase per MFMA.
template <int WAVES, int BNB, int MODE, bool UPS, bool SGB = false>
__global__ void __launch_bounds__(64 * WAVES, 1) conv_halo_kernel(const GemmArgs p, const HaloGeo g) {
  using T = HcT<WAVES, BNB>;
  constexpr int BN = T::BN, WN = T::WN, HJ = T::HJ, WJ = T::WJ, BMB = T::BMB;
  extern __shared__ __attribute__((aligned(16))) bf16_t hc_smem[];
  bf16_t* const halo = hc_smem;                                  // [2][HPIX_MAX][64]
  bf16_t* const wst = hc_smem + 2 * T::HALO_ELEMS;               // [2][BN][64]
  float* const ssb = reinterpret_cast<float*>(wst + 2 * T::W_ELEMS);  // [2][256]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid & 3, wc = wid >> 2;   // SIMD partners (w, w + 4) share rows, split the columns

  // ---- tile: XCD-contiguous block order, N-tile major (an XCD's workgroups stream one W slice through its L2)
  const int total = g.tiles_m * g.tiles_n;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = total >> 3, r = total & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int nt = bid / g.tiles_m, mt = bid - nt * g.tiles_m;
  const int m0 = mt * HC_BM, n0 = nt * BN;
  const int tpi = p.OH / g.TR;                 // tiles per image
  const int img = mt / tpi, row0 = (mt - img * tpi) * g.TR;

  const int cs_a = p.A2 ? p.Cin1 : p.Cin, cs_b = p.Cin - p.Cin1;
  const long src_pix = (long)p.Nimg * p.H * p.Wd;
  const __amdgpu_buffer_rsrc_t rA = hc_rsrc(p.A, src_pix * cs_a * 2);
  const __amdgpu_buffer_rsrc_t rA2 = p.A2 ? hc_rsrc(p.A2, src_pix * cs_b * 2) : rA;
  const __amdgpu_buffer_rsrc_t rW = hc_rsrc(p.W, (long)p.N * p.ldw * 2);
  // scale and shift are one allocation (host-checked): shift = scale + Nimg * Cin
  const __amdgpu_buffer_rsrc_t rS = MODE ? hc_rsrc(p.in_scale, (long)2 * p.Nimg * p.Cin * 4) : rW;

  // ---- halo DMA geometry: instruction j of wave wid covers halo pixels (wid HJ + j) 8 + 0..7; lane -> pixel
  // P = ... + (lane >> 3), slot lane & 7 = logical chunk hcc ^ (P & 7) = hcc ^ (lane >> 3)
  const int hcc = (lane & 7) ^ (lane >> 3);
  int hsrc[HJ];   // source pixel of each of this lane's halo slots, -1: padding / past the halo (zero fill)
#pragma unroll
  for (int j = 0; j < HJ; ++j) {
    const int P = (wid * HJ + j) * 8 + (lane >> 3);
    const int hr = P / g.HC, hc = P - hr * g.HC;
    const int y = row0 - 1 + hr, x = hc - 1;
    const bool ok = P < g.HPIX && (unsigned)y < (unsigned)p.OH && (unsigned)x < (unsigned)p.OW;
    int src;
    if constexpr (UPS) src = (img * p.H + (y >> 1)) * p.Wd + (x >> 1);
    else src = (img * p.H + y) * p.Wd + x;
    hsrc[j] = ok ? src : -1;
  }
  auto dma_halo = [&](int c, int hb) {
    const int c0 = c * HC_BK;
    const bool second = p.A2 != nullptr && c0 >= p.Cin1;
    const uint32_t cs = (uint32_t)(second ? cs_b : cs_a);
    const uint32_t cb = (uint32_t)((second ? c0 - p.Cin1 : c0) + hcc * 8);
    bf16_t* base = halo + hb * T::HALO_ELEMS + wid * HJ * 8 * HC_BK;
#pragma unroll
    for (int j = 0; j < HJ; ++j) {
      const uint32_t off = hsrc[j] >= 0 ? ((uint32_t)hsrc[j] * cs + cb) * 2u : HC_OOB;
      SHAI_DASSERT_DMA(off, src_pix * cs * 2, HC_OOB);
      SHAI_DASSERT((wid * HJ + j + 1) * 8 <= HC_HPIX_MAX);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(second ? rA2 : rA, (hc_lds_void*)(base + j * 8 * HC_BK), 16, off, 0, 0,
                                               0);
    }
  };
  // scale / shift of the chunk's 64 channels for this image: lanes 0-15 scale, 16-31 shift, the rest zero fill
  auto dma_ss = [&](int c, int sb) {
    if constexpr (MODE != 0) {
      if (wid == 0) {
        uint32_t off = HC_OOB;
        if (lane < 32)
          off = (uint32_t)(((lane >= 16 ? p.Nimg * p.Cin : 0) + img * p.Cin + c * HC_BK + (lane & 15) * 4) * 4);
        SHAI_DASSERT_DMA(off, (long)2 * p.Nimg * p.Cin * 4, HC_OOB);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rS, (hc_lds_void*)(ssb + sb * T::SS_FLOATS), 16, off, 0, 0, 0);
      }
    }
  };

  // ---- W DMA: stage row r = output column n0 + r; its 16-B slot s holds K chunk s ^ ((r >> 1) & 7)
  uint32_t woff[WJ];
#pragma unroll
  for (int u = 0; u < WJ; ++u) {
    const int r = (wid + WAVES * u) * 8 + (lane >> 3);
    const int n = n0 + r;
    woff[u] = (r < BN && n < p.N) ? (uint32_t)(((long)n * p.ldw + (((lane & 7) ^ ((r >> 1) & 7)) * 8)) * 2) : HC_OOB;
  }
  const int nk = 9 * g.nchunks;
  auto dma_w = [&](int t, int st) {
    const int c = t / 9, tap = t - 9 * c;
    const uint32_t koff = (uint32_t)((tap * p.Cin + c * HC_BK) * 2);
    bf16_t* base = wst + st * T::W_ELEMS;
#pragma unroll
    for (int u = 0; u < WJ; ++u) {
      const int q = wid + WAVES * u;
      // (the offset is computed into a variable: a conditional expression as the builtin's argument silently
      // drops the host-side kernel stub -- the .o then references an undefined __device_stub__)
      const uint32_t off = woff[u] == HC_OOB ? HC_OOB : woff[u] + koff;
      SHAI_DASSERT_DMA(off, (long)p.N * p.ldw * 2, HC_OOB);
      SHAI_DASSERT(t < nk && st >= 0 && st < 2);
      if (q < BN / 8)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (hc_lds_void*)(base + q * 8 * HC_BK), 16, off, 0, 0, 0);
    }
  };

  // ---- normalisation of this lane's own halo slots of buffer hb with the scale / shift of slot sb: branch-free
  // (padding slots select 0, the DMA's zero fill; the whole step stays ONE basic block, so hipcc interleaves this
  // VALU work with the step's MFMAs).  silu(y) = y / (1 + 2^(-y log2 e)), y = x sc + sh: fma, mul, v_exp, add,
  // v_rcp, mul per element (per-chunk exp2 coefficients would save the mul but cost 16 registers: the 8-wave build
  // sits at the 256-register cap).
  float sc[8], sh[8];
  uint32_t hvalid = 0;   // bit j: this lane's halo slot j is a real pixel
#pragma unroll
  for (int j = 0; j < HJ; ++j) hvalid |= (hsrc[j] >= 0 ? 1u : 0u) << j;
  auto load_ss = [&](int sb) {
    const float* s = ssb + sb * T::SS_FLOATS;
    const float4_ a0 = *reinterpret_cast<const float4_*>(s + hcc * 8);
    const float4_ a1 = *reinterpret_cast<const float4_*>(s + hcc * 8 + 4);
    const float4_ b0 = *reinterpret_cast<const float4_*>(s + 64 + hcc * 8);
    const float4_ b1 = *reinterpret_cast<const float4_*>(s + 64 + hcc * 8 + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sc[e] = a0[e]; sc[4 + e] = a1[e];
      sh[e] = b0[e]; sh[4 + e] = b1[e];
    }
  };
  auto norm_slot = [&](int hb, int j) {
    uint4_* q = reinterpret_cast<uint4_*>(halo + hb * T::HALO_ELEMS + ((wid * HJ + j) * 8) * HC_BK) + lane;
    const uint4_ v = *q;
    float f[8];
    unpack8(v, f);
    const bool ok = (hvalid >> j) & 1u;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float y = fmaf(f[e], sc[e], sh[e]);
      const float ex = __builtin_amdgcn_exp2f(y * -1.4426950408889634f);
      f[e] = ok ? y * rcp_f(1.0f + ex) : 0.f;
    }
    *q = pack8(f);
  };

  // ---- fragments.  A: output pixel 64 wr + 16 i + fr of the tile = row r, column col -> halo pixel r HC + col at
  // tap (0, 0), + kh HC + kw at tap (kh, kw).  W: row wc WN + 16 j + fr of the stage.
  const int fr = lane & 15, fq = lane >> 4;
  int hp0[BMB];
#pragma unroll
  for (int i = 0; i < BMB; ++i) {
    const int ml = 64 * wr + 16 * i + fr;
    hp0[i] = (ml >> g.lg_ow) * g.HC + (ml & ((1 << g.lg_ow) - 1));
  }
  auto a_off = [&](int i, int ks, int tsh) {
    const int pp = hp0[i] + tsh;
    SHAI_DASSERT(pp >= 0 && pp < g.HPIX && g.HPIX <= HC_HPIX_MAX);
    return pp * HC_BK + (((4 * ks + fq) ^ (pp & 7)) << 3);
  };
  auto w_off = [&](int j, int ks) { return (wc * WN + 16 * j + fr) * HC_BK + (((4 * ks + fq) ^ ((fr >> 1) & 7)) << 3); };

  float4_ acc[BMB][BNB];
  hcbf16x8 x0[BMB], w0[BNB], x1[BMB], w1[BNB];
  auto tile_tsh = [&](int t) {
    const int tap = t - 9 * (t / 9);
    const int kh = tap / 3;
    return kh * g.HC + (tap - 3 * kh);
  };
  auto read_frags = [&](int t, int ks, hcbf16x8* xs, hcbf16x8* ws) {
    const bf16_t* hb = halo + ((t / 9) & 1) * T::HALO_ELEMS;
    const bf16_t* wb = wst + (t & 1) * T::W_ELEMS;
    const int tsh = tile_tsh(t);
#pragma unroll
    for (int j = 0; j < BNB; ++j) ws[j] = *reinterpret_cast<const hcbf16x8*>(wb + w_off(j, ks));
#pragma unroll
    for (int i = 0; i < BMB; ++i) xs[i] = *reinterpret_cast<const hcbf16x8*>(hb + a_off(i, ks, tsh));
  };

  // ---- prologue: chunk 0's halo (+ scale / shift), W tiles 0 and 1
  dma_halo(0, 0);
  dma_ss(0, 0);
  dma_w(0, 0);
  if (nk > 1) dma_w(1, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();   // scale / shift (wave 0's DMA) visible to every wave
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (MODE != 0) {
    load_ss(0);
#pragma unroll
    for (int j = 0; j < HJ; ++j) norm_slot(0, j);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  read_frags(0, 0, x0, w0);

  // The main loop walks the chunks with the 9 taps unrolled, so every per-tap decision is compile-time and a step is
  // one basic block: the next chunk's normalisation slots (taps 1..7; its DMA was issued at tap 0 and waited for by
  // tap 1's vmcnt(0)) interleave with the step's MFMAs.  Past the last chunk / tile the DMAs re-load the last valid
  // chunk / tile and the normalisation runs over the idle halo buffer: harmless (never read), and no branch.
  constexpr int NPT = (HJ + 6) / 7;
  auto seg_a = [&](int t, bool first) {
    read_frags(t, 1, x1, w1);
    const float4_ z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < BMB; ++i)
#pragma unroll
      for (int j = 0; j < BNB; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[j], x0[i], first ? z : acc[i][j], 0, 0, 0);
  };
  auto seg_bc = [&](int c, auto tap_c) {
    constexpr int TAP = decltype(tap_c)::value;
    const int t = 9 * c + TAP;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < BMB; ++i) asm volatile("" : "+v"(x1[i]));
#pragma unroll
    for (int j = 0; j < BNB; ++j) asm volatile("" : "+v"(w1[j]));
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const int cn = min(c + 1, g.nchunks - 1);   // the next chunk (the last one again past the end)
    dma_w(min(t + 2, nk - 1), t & 1);
    if constexpr (TAP == 0) {
      dma_halo(cn, (c + 1) & 1);
      dma_ss(cn, (c + 1) & 1);
    }
    constexpr bool NORM_STEP = MODE != 0 && TAP >= 1 && TAP <= 7;
    if constexpr (SGB && NORM_STEP) {
      // hand-interleaved normalisation (lab variant): this step's NPT slots (16 elements each as two 3-op phases:
      // y = fma, e = exp2(-y log2 e) | o = y / (1 + e)) one phase per MFMA, order pinned by sched_barrier; the raw
      // slots are read BEFORE the next tile's fragments (LDS returns in order: their wait does not cover those)
      if constexpr (TAP == 1) load_ss((c + 1) & 1);
      const int hb = (c + 1) & 1;
      uint4_* qs[NPT];
      uint4_ raw[NPT];
#pragma unroll
      for (int u = 0; u < NPT; ++u) {
        const int j = min((TAP - 1) * NPT + u, HJ - 1);
        qs[u] = reinterpret_cast<uint4_*>(halo + hb * T::HALO_ELEMS + ((wid * HJ + j) * 8) * HC_BK) + lane;
        raw[u] = *qs[u];
      }
      read_frags(min(t + 1, nk - 1), 0, x0, w0);
      float f[NPT][8], yv[NPT][8], ev[NPT][8];
      constexpr int NSTG = 16 * NPT;
      static_assert(NSTG <= BMB * BNB, "normalisation phases per step");
#pragma unroll
      for (int i = 0; i < BMB; ++i)
#pragma unroll
        for (int j = 0; j < BNB; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[j], x1[i], acc[i][j], 0, 0, 0);
          const int k = i * BNB + j;
          if (k < NSTG) {
            const int u = k / 16, e = (k % 16) >> 1;
            if ((k & 1) == 0) {
              if (e == 0) unpack8(raw[u], f[u]);
              yv[u][e] = fmaf(f[u][e], sc[e], sh[e]);
              ev[u][e] = __builtin_amdgcn_exp2f(yv[u][e] * -1.4426950408889634f);
            } else {
              const int jj = (TAP - 1) * NPT + u;
              const bool ok = jj < HJ && ((hvalid >> min(jj, HJ - 1)) & 1u);
              f[u][e] = ok ? yv[u][e] * rcp_f(1.0f + ev[u][e]) : 0.f;
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
      for (int u = 0; u < NPT; ++u)
        if ((TAP - 1) * NPT + u < HJ) *qs[u] = pack8(f[u]);
    } else {
      read_frags(min(t + 1, nk - 1), 0, x0, w0);
      if constexpr (MODE != 0 && TAP == 1) load_ss((c + 1) & 1);
#pragma unroll
      for (int i = 0; i < BMB; ++i)
#pragma unroll
        for (int j = 0; j < BNB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[j], x1[i], acc[i][j], 0, 0, 0);
      if constexpr (NORM_STEP) {
#pragma unroll
        for (int u = 0; u < NPT; ++u)
          if ((TAP - 1) * NPT + u < HJ) norm_slot((c + 1) & 1, (TAP - 1) * NPT + u);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < BMB; ++i) asm volatile("" : "+v"(x0[i]));
#pragma unroll
    for (int j = 0; j < BNB; ++j) asm volatile("" : "+v"(w0[j]));
  };
  auto step = [&](int c, auto tap_c) {   // seg_bc(t) then seg_a(t + 1)
    constexpr int TAP = decltype(tap_c)::value;
    seg_bc(c, tap_c);
    if (TAP < 8 || c + 1 < g.nchunks) seg_a(9 * c + TAP + 1, false);
  };

  seg_a(0, true);
  for (int c = 0; c < g.nchunks; ++c) {
    step(c, std::integral_constant<int, 0>{});
    step(c, std::integral_constant<int, 1>{});
    step(c, std::integral_constant<int, 2>{});
    step(c, std::integral_constant<int, 3>{});
    step(c, std::integral_constant<int, 4>{});
    step(c, std::integral_constant<int, 5>{});
    step(c, std::integral_constant<int, 6>{});
    step(c, std::integral_constant<int, 7>{});
    step(c, std::integral_constant<int, 8>{});
  }
  // every LDS-DMA (the re-loads past the end included) has landed before the epilogue reuses the LDS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- epilogue (host: M % 256 == 0, N % BN == 0, 16-B aligned operands, ldc = ldr = N): lane owns pixel
  // m0 + 64 wr + 16 i + fr and columns n0 + wc WN + 16 j + 4 fq .. + 3
  const bf16_t* R = p.residual;
  float bj[BNB][4];
#pragma unroll
  for (int j = 0; j < BNB; ++j) {
    const int n = n0 + wc * WN + 16 * j + 4 * fq;
#pragma unroll
    for (int e = 0; e < 4; ++e) bj[j][e] = 0.f;
    if (p.bias) {
      const uint2_ bb = *reinterpret_cast<const uint2_*>(p.bias + n);
      bj[j][0] = bf2f(bb[0] & 0xffff); bj[j][1] = bf2f(bb[0] >> 16);
      bj[j][2] = bf2f(bb[1] & 0xffff); bj[j][3] = bf2f(bb[1] >> 16);
    }
    if (p.bias2d) {  // the tile lies in one image: one time-embedding row
      const uint2_ bb = *reinterpret_cast<const uint2_*>(p.bias2d + (long)img * p.N + n);
      bj[j][0] += bf2f(bb[0] & 0xffff); bj[j][1] += bf2f(bb[0] >> 16);
      bj[j][2] += bf2f(bb[1] & 0xffff); bj[j][3] += bf2f(bb[1] >> 16);
    }
  }
  float cs[BNB][4], cq[BNB][4];   // column partials of the stored (bf16-rounded) output over this lane's rows
#pragma unroll
  for (int j = 0; j < BNB; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) cs[j][e] = cq[j][e] = 0.f;
  const bool stats = p.col_part != nullptr;
#pragma unroll
  for (int i = 0; i < BMB; ++i) {
    const long m = m0 + 64 * wr + 16 * i + fr;
    uint2_ rr[BNB];
    if (R) {
#pragma unroll
      for (int j = 0; j < BNB; ++j)
        rr[j] = *reinterpret_cast<const uint2_*>(R + m * p.ldr + n0 + wc * WN + 16 * j + 4 * fq);
    }
#pragma unroll
    for (int j = 0; j < BNB; ++j) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bj[j][e];
      if (R) {
        v[0] += bf2f(rr[j][0] & 0xffff) * p.res_alpha; v[1] += bf2f(rr[j][0] >> 16) * p.res_alpha;
        v[2] += bf2f(rr[j][1] & 0xffff) * p.res_alpha; v[3] += bf2f(rr[j][1] >> 16) * p.res_alpha;
      }
      uint2_ o;
      o[0] = pack2(v[0], v[1]);
      o[1] = pack2(v[2], v[3]);
      *reinterpret_cast<uint2_*>(p.C + m * p.ldc + n0 + wc * WN + 16 * j + 4 * fq) = o;
      if (stats) {
        const float f[4] = {bf2f(o[0] & 0xffff), bf2f(o[0] >> 16), bf2f(o[1] & 0xffff), bf2f(o[1] >> 16)};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          cs[j][e] += f[e];
          cq[j][e] = fmaf(f[e], f[e], cq[j][e]);
        }
      }
    }
  }
  if (stats) {
    // sum over the 16 row lanes (fr) of each column quad, then the two waves of a 128-row block meet in LDS
#pragma unroll
    for (int j = 0; j < BNB; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          cs[j][e] += __shfl_xor(cs[j][e], o, 64);
          cq[j][e] += __shfl_xor(cq[j][e], o, 64);
        }
    float* red = reinterpret_cast<float*>(hc_smem);   // [2 blocks][BN][2]: the halo buffer, free after the loop
    __syncthreads();
    if ((wr & 1) && fr == 0) {
#pragma unroll
      for (int j = 0; j < BNB; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = wc * WN + 16 * j + 4 * fq + e;
          red[((wr >> 1) * BN + col) * 2] = cs[j][e];
          red[((wr >> 1) * BN + col) * 2 + 1] = cq[j][e];
        }
    }
    __syncthreads();
    if (!(wr & 1) && fr == 0) {
      float* cp = p.col_part + ((long)((m0 >> 7) + (wr >> 1)) * p.N + n0) * 2;
#pragma unroll
      for (int j = 0; j < BNB; ++j) {
        const int col = wc * WN + 16 * j + 4 * fq;
        const float* rv = red + ((wr >> 1) * BN + col) * 2;
        float4_ lo = {cs[j][0] + rv[0], cq[j][0] + rv[1], cs[j][1] + rv[2], cq[j][1] + rv[3]};
        float4_ hi = {cs[j][2] + rv[4], cq[j][2] + rv[5], cs[j][3] + rv[6], cq[j][3] + rv[7]};
        *reinterpret_cast<float4_*>(cp + col * 2) = lo;
        *reinterpret_cast<float4_*>(cp + col * 2 + 4) = hi;
      }
    }
  }
}

// ---------------------------------------------------------------------------- host side
static bool hc_al16(const void* q) { return ((uintptr_t)q & 15) == 0; }

static int hc_bn(const GemmArgs& a) { return a.N % 160 == 0 ? 160 : (a.N % 128 == 0 ? 128 : 0); }

bool conv_halo_supported(const GemmArgs& a) {
  if (!a.conv || a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad != 1 || a.batch > 1) return false;
  if (a.OW != 16 && a.OW != 32 && a.OW != 64) return false;
  const int TR = HC_BM / a.OW;
  if (a.OH % TR != 0 || (TR + 2) * (a.OW + 2) > HC_HPIX_MAX) return false;
  if (a.M != a.Nimg * a.OH * a.OW || a.M % HC_BM != 0) return false;
  if (a.Cin % 64 != 0 || (a.A2 != nullptr && (a.Cin1 % 64 != 0 || a.Cin1 <= 0))) return false;
  if (hc_bn(a) == 0) return false;
  if (a.act != ACT_NONE || a.glu || a.gate || a.rms || a.w_scale || a.row_mr || a.alpha != 1.f) return false;
  if (a.in_scale != nullptr) {
    // GroupNorm + SiLU (the only normalised variant instantiated); scale and shift in one allocation
    if (a.in_act != ACT_SILU || a.upsample || a.in_shift != a.in_scale + (long)a.Nimg * a.Cin) return false;
    if (!hc_al16(a.in_scale) || a.Cin % 4 != 0) return false;
  }
  if (a.upsample == 2) return false;  // phase-decomposed upsample conv: v4 only
  if (a.upsample && (a.OH != 2 * a.H || a.OW != 2 * a.Wd)) return false;
  if (!a.upsample && (a.OH != a.H || a.OW != a.Wd)) return false;
  if (a.ldw != a.K || a.ldc != a.N || (a.residual && a.ldr != a.N)) return false;
  if (!hc_al16(a.A) || !hc_al16(a.W) || !hc_al16(a.C) || (a.A2 && !hc_al16(a.A2)) ||
      (a.residual && !hc_al16(a.residual)) || (a.bias && !hc_al16(a.bias)) || (a.bias2d && !hc_al16(a.bias2d)))
    return false;
  if (a.bias2d && a.rows_per_bias2d != a.OH * a.OW) return false;
  const long src_pix = (long)a.Nimg * a.H * a.Wd;
  const int cs_a = a.A2 ? a.Cin1 : a.Cin;
  if (src_pix * cs_a * 2 >= 0x7fffffffL || (a.A2 && src_pix * (a.Cin - a.Cin1) * 2 >= 0x7fffffffL)) return false;
  if ((long)a.N * a.ldw * 2 >= 0x7fffffffL) return false;
  return true;
}

template <int WAVES, int BNB, int MODE, bool UPS, bool SGB = false>
static void hc_go(const GemmArgs& a, const HaloGeo& g, hipStream_t s) {
  using T = HcT<WAVES, BNB>;
  conv_halo_kernel<WAVES, BNB, MODE, UPS, SGB><<<g.tiles_m * g.tiles_n, 64 * WAVES, T::LDS, s>>>(a, g);
}

template <int WAVES, int BNB, bool SGB = false>
static void hc_mode(const GemmArgs& a, const HaloGeo& g, hipStream_t s) {
  if (a.in_scale) hc_go<WAVES, BNB, 2, false, SGB>(a, g, s);
  else if (a.upsample) hc_go<WAVES, BNB, 0, true>(a, g, s);
  else hc_go<WAVES, BNB, 0, false>(a, g, s);
}

static int hc_waves_env() {
  static const int w = [] {
    const char* e = getenv("SHAI_HALO_WAVES");
    return (e && atoi(e) == 4) ? 4 : 8;
  }();
  return w;
}

void launch_conv_halo(const GemmArgs& a, hipStream_t s, int waves) {
  HaloGeo g;
  g.TR = HC_BM / a.OW;
  g.HC = a.OW + 2;
  g.HPIX = (g.TR + 2) * g.HC;
  g.lg_ow = a.OW == 16 ? 4 : (a.OW == 32 ? 5 : 6);
  const int bn = hc_bn(a);
  g.tiles_m = a.M / HC_BM;
  g.tiles_n = a.N / bn;
  g.nchunks = a.Cin / HC_BK;
  if (waves <= 0) waves = hc_waves_env();
  if (waves == 4) {
    if (bn == 160) hc_mode<4, 10>(a, g, s);
    else hc_mode<4, 8>(a, g, s);
  } else if (waves == 9) {  // lab: 8 waves with the normalisation hand-interleaved between the MFMAs
    if (bn == 160) hc_mode<8, 5, true>(a, g, s);
    else hc_mode<8, 4, true>(a, g, s);
  } else {
    if (bn == 160) hc_mode<8, 5>(a, g, s);
    else hc_mode<8, 4>(a, g, s);
  }
}

}  // namespace shai
