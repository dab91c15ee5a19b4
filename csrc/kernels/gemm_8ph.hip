// bf16 GEMM / implicit-GEMM convolution, v4: 8-phase ping-pong schedule, 256x256 / 256x320 tile, BK = 64.
//
//   C[b,m,n] = gate * act(alpha * sum_k A[b,m,k] * W[b,n,k] + bias[n] + bias2d) + res_alpha * Res[b,m,n]
//
// Why a fourth kernel: v3 (the pipelined gemm_pipe.hip, retired in round 5) kept several K-tiles of LDS-DMA in flight, but every K-step
// still starts with all 8 waves issuing their fragment reads at once, so each SIMD's matrix pipe idles
// for the LDS latency of both of its waves once per 32-deep step (measured 1.08-1.2 PF on large plain
// GEMMs vs 1.5-1.6 PF for hipBLASLt).  Here the two waves that share a SIMD run half a phase apart:
//
// * 8 waves = 2 groups (waves 0-3 and 4-7; wave w and w+4 share a SIMD).  Group 1 executes one extra
//   s_barrier up front, so while one group runs its 16-MFMA "compute" segment the other runs its
//   "load" segment (fragment ds_reads + LDS-DMA issue), and the roles swap at every barrier.  The
//   matrix pipe of each SIMD sees back-to-back MFMA segments from alternating waves.
// * 256 x BN output tile (BN = 256, or 320: every SD2.1 UNet channel count is a multiple of 320), each
//   wave 128 (M) x BN/4 (N) = 8 x NJ blocks of v_mfma_f32_16x16x32_bf16 (NJ = 4 / 5) with the W
//   fragment as the A operand (each lane owns 4 consecutive output columns of one row).
// * A K-tile (64 deep) is 4 phases: (k-substep 0|1) x (M half 0|1), 4 x NJ MFMAs each.  W fragments
//   (NJ ds_read_b128) are read in the first phase of each k-substep and held for the second; X
//   fragments (4 ds_read_b128) are read every phase.
// * 2 LDS buffers of (A 256x64 + W BNx64) bf16 = 128 / 144 KB.  Tile t+1 is staged into the other
//   buffer by LDS-DMA (`buffer_load ... lds`, 16 B per lane; 4 A + NJ W instructions per wave per
//   K-tile, A and W interleaved) over phases 0-1 of tile t; every wave retires its own DMA with vmcnt(0)
//   at the end of its phase-3 load segment, which precedes (in barrier order) every wave's first read
//   of tile t+1.
// * Each load segment ends with lgkmcnt(0) BEFORE its barrier, so when a group starts restaging a
//   buffer the other group's reads of it have completed (WAR across the half-phase stagger).
// * LDS image lane-linear per DMA wave-instruction (8 rows x 128 B); bank swizzle (16-B chunk ^=
//   (row >> 1) & 7) applied to the per-lane SOURCE address and to the ds_read address: every 16-lane
//   ds_read_b128 group touches 16 distinct 16-B bank slots (conflict-free).
// * Implicit-GEMM conv when Cin (and the concat split Cin1) are multiples of 64: each K-tile then lies
//   inside one filter tap and one source tensor, so only (ih, iw) of the lane's 4 rows change per tile.
// * Range-checked buffer descriptors give the zero fill (M/N/K tails, conv padding); XCD-aware
//   bijective block remap + grouped M ordering.
// * Persistent form (VAR bit 3, configs kV4Cfg + 2 / + 3): one workgroup per CU walks output tiles
//   blockIdx.x + i * gridDim.x (gridDim.x % 8 == 0 keeps every tile of a workgroup on its XCD).  After
//   a tile's last K-step both LDS buffers are free, so the first K-tile of the NEXT tile is put in flight
//   before this tile's epilogue runs: on low-K problems (K = 320..1280, 5-20 K-tiles) the
//   epilogue's residual reads / activation / stores overlap the next tile's operand fetch instead of
//   leaving the matrix pipe idle for a full HBM round trip per tile.
#include "gemm_epilogue.h"

#include <algorithm>

namespace shai {

typedef __bf16 bf16x8q __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void g4_lds_void;

constexpr int G4_BM = 256, G4_BK = 64;
template <int BN>
struct G4T {
  static constexpr int STAGE = (G4_BM + BN) * G4_BK;  // elements per LDS buffer (64 / 72 KB)
  static constexpr int NJ = BN / 64;                   // 16-column MFMA blocks per wave (4 / 5)
  static constexpr int WC = BN / 4;                    // columns per wave (64 / 80)
  static constexpr int NWJ = BN / 64;                  // W DMA instructions (8 rows each) per wave per tile
  static constexpr int GT = 4 + NWJ;                   // DMA instructions per wave per tile
};
constexpr uint32_t G4_OOB = 0x80000000u;

__device__ __forceinline__ int g4_swz(int row, int ch) { return row * G4_BK + ((ch ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t g4_rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)min(bytes, 0x7fffffffL),
                                           0x00020000);
}

__device__ __forceinline__ void g4_glds(__amdgpu_buffer_rsrc_t r, bf16_t* lds, uint32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (g4_lds_void*)lds, 16, off, 0, 0, 0);
}

// Schedule variants (lab A/B; 0 = production):
//   bit 0: no stagger (both wave groups in lockstep)
//   bit 1: static priority (waves 4-7 at prio 1 for the whole loop) instead of per-segment setprio
//   bit 2: LDS-DMA issued over phases 0-1 (halves) instead of over phases 0-2 (quarter, half, quarter)
//   bit 3: persistent tile loop with the next tile's first K-tile prefetched under the epilogue
//   bit 4: wide epilogue (W rows permuted in pairs of 16-column MFMA blocks, see g4_wperm: 16-B stores)
// Phase p of a K-tile issues the DMA instructions g in [G_p, G_{p+1}) of the next tile.
template <int VAR, int GT>
struct G4Sched {
  static constexpr int G1 = (VAR & 4) ? (GT + 1) / 2 : GT / 4, G2 = (VAR & 4) ? GT : (3 * GT) / 4;
};

// Wide epilogue.  A lane of a v_mfma_f32_16x16x32 block owns 4 consecutive output columns (4 fq .. 4 fq + 3),
// so the plain epilogue issues one 8-byte store per block and row: 40 store instructions per lane per tile
// at BN = 320, and a low-K tile (K = 320: 5 K-steps) spends about as long in those stores as in its MFMAs
// (stores are priced per wave-instruction, MI355X_MICROARCH "attention epilogue store tail").  The W tile
// is therefore staged with its rows permuted inside each pair of 16-column blocks (2q, 2q + 1) of a wave:
// LDS row 16 (2q + h) + n holds output column 32 q + 8 (n >> 2) + 4 h + (n & 3).  The MFMA is unchanged;
// lane fq of block 2q + h now owns columns 32 q + 8 fq + 4 h .. + 3, i.e. the pair gives the lane 8
// consecutive columns: one 16-byte store (bias / residual loads widen the same way).  A fifth block
// (BN = 320) keeps the identity mapping.  The permutation lives only in the DMA source row address.
template <int BN>
__device__ __forceinline__ int g4_wperm(int r) {  // LDS row of the W tile -> tile-local output column
  constexpr int WC = BN / 4, NP = BN / 128;       // columns per wave, block pairs per wave
  const int g = r / WC, loc = r - g * WC;
  const int jb = loc >> 4, nn = loc & 15;
  return jb < 2 * NP ? g * WC + (jb >> 1) * 32 + (nn >> 2) * 8 + (jb & 1) * 4 + (nn & 3) : r;
}
// tile-local first column of the 4 that lane quad fq of MFMA block j owns (within the wave's WC columns)
template <int BN, bool WIDE>
__device__ __forceinline__ int g4_col(int j, int fq) {
  constexpr int NP = BN / 128;
  if constexpr (WIDE) return j < 2 * NP ? (j >> 1) * 32 + 8 * fq + 4 * (j & 1) : j * 16 + 4 * fq;
  else return j * 16 + 4 * fq;
}

// Scalar (wave-uniform) position of a K-tile inside the implicit-GEMM conv: filter tap (kh, kw) and
// channel base c (Cin % 64 == 0, so a 64-deep K-tile never straddles a tap or the concat split).
struct G4ConvPos {
  int kh, kw, c;
};

// CONV: 0 plain GEMM, 1 implicit-GEMM conv, 2 implicit-GEMM conv over a nearest-2x upsampled input,
// 3 the same upsample + 3x3 conv decomposed by output phase (GemmArgs::upsample == 2): an output pixel
// (2i + py, 2j + px) of the upsampled grid reads only 2 x 2 distinct source pixels (rows i - 1 + py + a, columns
// j - 1 + px + b), so each of the 4 phases is a 2 x 2 conv over the LOW-resolution input with its own summed
// weights ([4 phases][Cout][4 taps x Cin], ops.pack_up2_phase_weight): K = 4 Cin instead of 9 Cin, 2.25x fewer
// FLOPs.  GEMM rows are ordered (image, phase, i, j), so a 256-row tile (H W % 256 == 0) has one image and one
// phase (its weight slice), the GroupNorm partials' 128-row blocks stay inside one image, and the epilogue maps
// each row to its output pixel.
template <int CONV, bool GLU, int ACT, bool SPLITK, int VAR, int BN>
__global__ void __launch_bounds__(512) gemm4_kernel(const GemmArgs p, float* __restrict__ ws, int k_per_split) {
  constexpr bool STAGGER = !(VAR & 1), STATIC_PRIO = (VAR & 2) != 0, PERSIST = (VAR & 8) != 0 && !SPLITK;
  constexpr bool WIDE = (VAR & 16) != 0;
  constexpr int NP = WIDE ? BN / 128 : 0;  // 16-column block pairs per wave with 8 consecutive columns per lane
  constexpr int G4_STAGE = G4T<BN>::STAGE, NJ = G4T<BN>::NJ, WC = G4T<BN>::WC, NWJ = G4T<BN>::NWJ;
  constexpr int GT = G4T<BN>::GT;
  constexpr int G4_G0 = 0, G4_G1 = G4Sched<VAR, GT>::G1, G4_G2 = G4Sched<VAR, GT>::G2, G4_G3 = GT;
  extern __shared__ __attribute__((aligned(16))) bf16_t g4_smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;  // wm = ping-pong group = M half of the tile

  // ---- tile mapping (XCD remap + grouped M ordering)
  const int tiles_m = (p.M + G4_BM - 1) / G4_BM, tiles_n = (p.N + BN - 1) / BN;
  const int total = tiles_m * tiles_n;
  auto tile_origin = [&](int bid, int& tm0, int& tn0) {
    {
      const int xcd = bid & 7, q = total >> 3, r = total & 7;
      bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    }
    constexpr int GROUP = 8;
    const int group = bid / (GROUP * tiles_n);
    const int first_m = group * GROUP;
    const int gsize = min(tiles_m - first_m, GROUP);
    const int in_group = bid - group * GROUP * tiles_n;
    tm0 = (first_m + in_group % gsize) * G4_BM;
    tn0 = (in_group / gsize) * BN;
  };
  int vb = blockIdx.x;  // virtual block id of the current tile (persistent: + i * gridDim.x)
  int m0, n0;
  tile_origin(vb, m0, n0);
  const int b = SPLITK ? 0 : blockIdx.y;
  const int kz = SPLITK ? blockIdx.y : 0;
  const int k_begin = kz * k_per_split;
  const int k_end = min(p.K, k_begin + k_per_split);

  const bf16_t* A = p.A + (long)b * p.batch_a;
  const bf16_t* Wt = p.W + (long)b * p.batch_w;
  const long w_sets = CONV == 3 ? 4 : (p.w_slice_rows > 0 ? (p.M + p.w_slice_rows - 1) / p.w_slice_rows : 1);
  const __amdgpu_buffer_rsrc_t rW = g4_rsrc(Wt, (long)p.N * p.ldw * 2 * w_sets);
  __amdgpu_buffer_rsrc_t rA, rA2;
  if constexpr (CONV != 0) {
    rA = g4_rsrc(A, (long)p.Nimg * p.H * p.Wd * (p.A2 ? p.Cin1 : p.Cin) * 2);
    rA2 = p.A2 ? g4_rsrc(p.A2, (long)p.Nimg * p.H * p.Wd * (p.Cin - p.Cin1) * 2) : rA;
  } else {
    rA = g4_rsrc(A, (long)p.M * p.lda * 2);
    rA2 = rA;
  }

  // ---- staging geometry: DMA wave-instruction j fills 8 LDS rows x 128 B (lane-linear); the lane's
  // source chunk is the swizzled one.  Per-row byte offsets are precomputed; an invalid row's offset
  // carries the OOB bit, which survives the per-tile additions (< 2^31) and reads as zero fill.
  const int lrow0 = lane >> 3, lpos0 = lane & 7;
  int kch[4];            // k offset of the lane's source chunk within the K-tile (A rows)
  int kchw[NWJ];         // same for the W rows
  uint32_t woff[NWJ];    // W row byte offset + chunk
  uint32_t aoff[4];      // plain GEMM: A row byte offset + chunk
  int ih0[4], iw0[4];    // conv: top-left input tap position of the output pixel (upsampled grid for CONV 2)
  int pix[4];            // conv (CONV 1): pixel index of (ih0, iw0); CONV 2: n * H
  // per-tile row offsets for the tile at (m0, n0); cheap enough to recompute rather than hold live
  // across the persistent loop's epilogue
  auto setup = [&]() {
    int lrow = lrow0, lpos = lpos0;  // opaque copies: a repeated setup() is recomputed, not CSE'd and held live
    if constexpr (PERSIST) asm volatile("" : "+v"(lrow), "+v"(lpos));
#pragma unroll
    for (int j = 0; j < NWJ; ++j) kchw[j] = (lpos ^ (((wid * (BN / 8) + j * 8 + lrow) >> 1) & 7)) * 8;
#pragma unroll
    for (int j = 0; j < 4; ++j) kch[j] = (lpos ^ (((wid * 32 + j * 8 + lrow) >> 1) & 7)) * 8;
#pragma unroll
    for (int j = 0; j < NWJ; ++j) {
      const int r = wid * (BN / 8) + j * 8 + lrow;  // LDS row
      const int n = n0 + (WIDE ? g4_wperm<BN>(r) : r);
      // phase conv: the tile's phase selects its weight slice (rows ph N .. ph N + N - 1)
      // phase conv: the tile's phase selects its weight slice; w_slice_rows: the tile's row block does
      const long wrow = CONV == 3 ? (long)up2_row(p, m0).ph * p.N + n
                                  : (p.w_slice_rows > 0 ? (long)(m0 / p.w_slice_rows) * p.N + n : (long)n);
      woff[j] = n < p.N ? (uint32_t)((wrow * p.ldw + kchw[j]) * 2) : G4_OOB;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + wid * 32 + j * 8 + lrow;
      if constexpr (CONV == 0) {
        aoff[j] = m < p.M ? (uint32_t)(((long)m * p.lda + kch[j]) * 2) : G4_OOB;
      } else {
        const int hw = p.OH * p.OW;
        const int mm = m < p.M ? m : 0;
        const int cn = mm / hw;
        const int rem = mm - cn * hw;
        const int coh = rem / p.OW, cow = rem - coh * p.OW;
        if constexpr (CONV == 3) {
          // row (image, phase, i, j): 2 x 2 taps from source row i - 1 + py, column j - 1 + px
          const Up2Row q = up2_row(p, mm);
          ih0[j] = m < p.M ? q.si - 1 + (q.ph >> 1) : -(1 << 24);
          iw0[j] = q.sj - 1 + (q.ph & 1);
          pix[j] = (q.img * p.H + ih0[j]) * p.Wd + iw0[j];
          (void)cn;
          (void)coh;
          (void)cow;
        } else if constexpr (CONV == 1) {
          ih0[j] = m < p.M ? coh * p.stride - p.pad : -(1 << 24);
          iw0[j] = cow * p.stride - p.pad;
          pix[j] = (cn * p.H + ih0[j]) * p.Wd + iw0[j];
        } else {
          ih0[j] = m < p.M ? coh - p.pad : -(1 << 24);
          iw0[j] = cow - p.pad;
          pix[j] = cn * p.H;
        }
        aoff[j] = (uint32_t)kch[j] * 2;
      }
    }
  };
  setup();
  const int cs_a = p.A2 ? p.Cin1 : p.Cin;  // channel stride (elements per pixel) of source A / A2
  const int cs_b = p.Cin - p.Cin1;

  // Issue DMA g of the K-tile at k0 (conv position cp) into buffer buf: g < 8: even = A rows j = g / 2,
  // odd = W rows j = g / 2 (A and W interleave so every phase that stages issues both kinds); g = 8: W
  // rows 4 (BN = 320).
  auto stage_one = [&](int buf, int k0, const G4ConvPos& cp, int g) {
    bf16_t* sa = g4_smem + buf * G4_STAGE;
    const int j = g >> 1;
    const bool ktail = k0 + G4_BK > k_end;  // uniform: only the last K-tile of a ragged K checks chunks
    if ((g & 1) || g == 8) {
      uint32_t off = woff[j] + (uint32_t)k0 * 2;
      if (ktail && k0 + kchw[j] >= k_end) off = G4_OOB;
      SHAI_DASSERT_DMA(off, (long)p.N * p.ldw * 2 * w_sets, G4_OOB);
      SHAI_DASSERT(buf >= 0 && buf < 2);
      g4_glds(rW, sa + G4_BM * G4_BK + (wid * (BN / 8) + j * 8) * G4_BK, off);
      return;
    }
    if constexpr (CONV == 0) {
      uint32_t off = aoff[j] + (uint32_t)k0 * 2;
      if (ktail && k0 + kch[j] >= k_end) off = G4_OOB;
      SHAI_DASSERT_DMA(off, (long)p.M * p.lda * 2, G4_OOB);
      g4_glds(rA, sa + (wid * 32 + j * 8) * G4_BK, off);
    } else {
      const bool second = p.A2 != nullptr && cp.c >= p.Cin1;
      const int cs = second ? cs_b : cs_a;
      const int cb = second ? cp.c - p.Cin1 : cp.c;
      const int ih = ih0[j] + cp.kh, iw = iw0[j] + cp.kw;
      uint32_t off;
      if constexpr (CONV == 1 || CONV == 3) {
        const bool ok = ((unsigned)ih < (unsigned)p.H) & ((unsigned)iw < (unsigned)p.Wd);
        const int tapd = cp.kh * p.Wd + cp.kw;
        off = ok ? (uint32_t)((pix[j] + tapd) * cs + cb) * 2 + aoff[j] : G4_OOB;
      } else {
        const bool ok = ((unsigned)ih < (unsigned)(2 * p.H)) & ((unsigned)iw < (unsigned)(2 * p.Wd));
        const int px = (pix[j] + (ih >> 1)) * p.Wd + (iw >> 1);
        off = ok ? (uint32_t)(px * cs + cb) * 2 + aoff[j] : G4_OOB;
      }
      if (k0 >= k_end) off = G4_OOB;
      SHAI_DASSERT_DMA(off, (long)p.Nimg * p.H * p.Wd * cs * 2, G4_OOB);
      g4_glds(second ? rA2 : rA, sa + (wid * 32 + j * 8) * G4_BK, off);
    }
  };
  auto conv_pos = [&](int k0) {
    G4ConvPos cp{0, 0, 0};
    if constexpr (CONV != 0) {
      const int tap = k0 / p.Cin;
      cp.c = k0 - tap * p.Cin;
      cp.kh = tap / p.KW;
      cp.kw = tap - cp.kh * p.KW;
    }
    return cp;
  };
  auto conv_advance = [&](G4ConvPos& cp) {
    if constexpr (CONV != 0) {
      cp.c += G4_BK;
      if (cp.c >= p.Cin) {
        cp.c = 0;
        if (++cp.kw == p.KW) {
          cp.kw = 0;
          ++cp.kh;
        }
      }
    }
  };

  const int fr = lane & 15, fq = lane >> 4;
  const int nk = k_end > k_begin ? (k_end - k_begin + G4_BK - 1) / G4_BK : 0;

  // prologue: K-tile 0 of the first output tile -> buffer 0
  G4ConvPos cpos = conv_pos(k_begin);
  if (nk > 0) {
#pragma unroll
    for (int g = 0; g < GT; ++g) stage_one(0, k_begin, cpos, g);
  }
  bf16x8q wf[NJ], xf[4];
  // VAR bit 5 (persistent only): the wide epilogue's stores stay in flight into the next tile.  The top of
  // the loop then waits only for the next tile's first K-tile (DMA issued BEFORE the epilogue): vmcnt
  // counts in issue order, and the fast wide epilogue issues at least G4_NOUT vector-memory instructions
  // (its stores) after that DMA.  Any other epilogue path drains with vmcnt(0) below.
  constexpr bool NODRAIN = (VAR & 32) != 0 && PERSIST && WIDE;
  constexpr int G4_NOUT = 8 * (NP + (2 * NP < NJ ? 1 : 0));
  static_assert(G4_NOUT < 63, "vmcnt range");
  bool first = true, wide_done = false;
  while (true) {
    if (!NODRAIN || first || !wide_done) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G4_NOUT) : "memory");
    first = false;
    wide_done = false;
    __builtin_amdgcn_s_barrier();
    if (STAGGER && wm == 1) __builtin_amdgcn_s_barrier();  // stagger: group 1 runs half a phase behind
    if (STATIC_PRIO && wm == 1) __builtin_amdgcn_s_setprio(1);
    __builtin_amdgcn_sched_barrier(0);

    float4_ acc[8][NJ];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = float4_{0.f, 0.f, 0.f, 0.f};
    // fragment-read lane coordinates made opaque per output tile: the ds_read addresses derived from them
    // are then rebuilt per tile instead of being hoisted out of the persistent loop and held live
    // (about 30 registers) across the epilogue
    int frl = fr, fql = fq;
    if constexpr (PERSIST) asm volatile("" : "+v"(frl), "+v"(fql));

    for (int t = 0; t < nk; ++t) {
      const int cur = t & 1;
      const bool pre = t + 1 < nk;
      const int knext = k_begin + (t + 1) * G4_BK;
      conv_advance(cpos);  // position of tile t + 1
      const bf16_t* sa = g4_smem + cur * G4_STAGE;
      const bf16_t* sw = sa + G4_BM * G4_BK;
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) {
        const int ks = ph >> 1, mh = ph & 1;
        // ---- load segment
        const int g_lo = ph == 0 ? G4_G0 : ph == 1 ? G4_G1 : ph == 2 ? G4_G2 : G4_G3;
        const int g_hi = ph == 0 ? G4_G1 : ph == 1 ? G4_G2 : ph == 2 ? G4_G3 : GT;
        if (pre) {
#pragma unroll
          for (int g = g_lo; g < g_hi; ++g) stage_one(cur ^ 1, knext, cpos, g);
        }
        if (mh == 0) {
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            wf[j] = *reinterpret_cast<const bf16x8q*>(sw + g4_swz(wn * WC + j * 16 + frl, ks * 4 + fql));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          xf[i] = *reinterpret_cast<const bf16x8q*>(sa + g4_swz(wm * 128 + (mh * 4 + i) * 16 + frl, ks * 4 + fql));
        if (ph == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile t+1 landed
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        // ---- compute segment
        if (!STATIC_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[mh * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[mh * 4 + i][j], 0, 0, 0);
        if (!STATIC_PRIO) __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (STATIC_PRIO) __builtin_amdgcn_s_setprio(0);
    if (STAGGER && wm == 0) __builtin_amdgcn_s_barrier();  // un-stagger: equal barrier counts on exit

    // every wave is past its last LDS read of this tile (lgkmcnt(0) precedes each load-segment barrier):
    // both buffers are free, so the next tile's first K-tile goes in flight under this epilogue
    const int em0 = m0, en0 = n0;
    bool more = false;
    if constexpr (PERSIST) {
      more = vb + (int)gridDim.x < total;
      if (more) {
        vb += gridDim.x;
        tile_origin(vb, m0, n0);
        setup();
        cpos = conv_pos(k_begin);
#pragma unroll
        for (int g = 0; g < GT; ++g) stage_one(0, k_begin, cpos, g);
        if constexpr (NODRAIN) {  // pin the DMA ahead of the epilogue's loads and stores (vmcnt order)
          asm volatile("" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    auto epilogue = [&, fr0 = fr, fq0 = fq](const int m0, const int n0) {
      // opaque lane coordinates: the epilogue's per-lane addressing is built here, not hoisted above the
      // persistent loop's main loop where it would pin registers for the whole K sweep
      int fr = fr0, fq = fq0;
      if constexpr (PERSIST) asm volatile("" : "+v"(fr), "+v"(fq));
      // ---- epilogue: D[n][m] blocks -> lane owns row m = fr, columns n..n+3 = 4 fq + reg
      if constexpr (SPLITK) {
        float* Wp = ws + (long)kz * p.M * p.N;
    #pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int m = m0 + wm * 128 + i * 16 + fr;
          if (m >= p.M) continue;
    #pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int n = n0 + wn * WC + g4_col<BN, WIDE>(j, fq);
            if (n + 3 < p.N) {
              *reinterpret_cast<float4_*>(Wp + (long)m * p.N + n) = acc[i][j];
            } else {
              for (int e = 0; e < 4 && n + e < p.N; ++e) Wp[(long)m * p.N + n + e] = acc[i][j][e];
            }
          }
        }
      } else {
        bf16_t* __restrict__ C = p.C + (long)b * p.batch_c;
        const bf16_t* __restrict__ R = p.residual ? p.residual + (long)b * p.batch_r : nullptr;
        // output row of GEMM row m: itself, or (phase conv) its pixel on the upsampled grid -- shifts and masks only
        // (up2_row): a division per row bloats the unrolled epilogue until the accumulators leave registers
        const auto orow = [&](int m) -> long {
          if constexpr (CONV == 3) return up2_out_row(p, m);
          else return m;
        };
        if (p.row_mr != nullptr) {
          // LayerNorm folded in (host: batch 1, unsplit): acc <- rstd[m] * (acc - mean[m] * s[n]), i.e. the GEMM of
          // the normalised rows with the gain-folded W; the folded shift is in the bias
          float mean[8], rstd[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int m = min(m0 + wm * 128 + i * 16 + fr, p.M - 1);
            const float2 v = *reinterpret_cast<const float2*>(p.row_mr + 2 * (long)m);
            mean[i] = v.x;
            rstd[i] = v.y;
          }
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int n = n0 + wn * WC + g4_col<BN, WIDE>(j, fq);
            float s[4];
            if (n + 3 < p.N) {
              const float4_ sv = *reinterpret_cast<const float4_*>(p.col_s + n);
#pragma unroll
              for (int e = 0; e < 4; ++e) s[e] = sv[e];
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) s[e] = n + e < p.N ? p.col_s[n + e] : 0.f;
            }
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
              for (int e = 0; e < 4; ++e) acc[i][j][e] = rstd[i] * fmaf(-mean[i], s[e], acc[i][j][e]);
          }
        }
        // per-image bias (time embedding) in the wide path: each wave's 128 rows lie inside one image
        const bool b2ok = p.bias2d == nullptr ||
                          (WIDE && (p.rows_per_bias2d & 127) == 0 && (p.N & 7) == 0 && ((uintptr_t)p.bias2d & 15) == 0);
        const bool fast = m0 + G4_BM <= p.M && n0 + BN <= p.N && b2ok && p.gate == nullptr &&
                          (p.ldc & 3) == 0 && (R == nullptr || (p.ldr & 3) == 0);
        if constexpr (WIDE) {
          // 16-byte C / residual / bias accesses: 8-element aligned rows and bases
          const bool wide = fast && (((p.ldc | (R ? p.ldr : 0)) & 7) == 0) &&
                            ((((uintptr_t)C) | (uintptr_t)R | (uintptr_t)p.bias) & 15) == 0;
          if (wide) {
            const bf16_t* __restrict__ bias = p.bias;
            float bq[NP][8];
#pragma unroll
            for (int q = 0; q < NP; ++q) {
              const int n = n0 + wn * WC + q * 32 + 8 * fq;
              if (bias) unpack8(*reinterpret_cast<const uint4_*>(bias + n), bq[q]);
              else
#pragma unroll
                for (int e = 0; e < 8; ++e) bq[q][e] = 0.f;
            }
            constexpr bool TAIL = 2 * NP < NJ;  // BN = 320: block 4 keeps 4 columns per lane
            float bt[4] = {0.f, 0.f, 0.f, 0.f};
            const int nt4 = n0 + wn * WC + 2 * NP * 16 + 4 * fq;
            if (TAIL && bias) {
              const uint2_ bb = *reinterpret_cast<const uint2_*>(bias + nt4);
              bt[0] = bf2f(bb[0] & 0xffff); bt[1] = bf2f(bb[0] >> 16);
              bt[2] = bf2f(bb[1] & 0xffff); bt[3] = bf2f(bb[1] >> 16);
            }
            if (p.bias2d != nullptr) {  // b2ok: the wave's 128 rows share one bias2d row
              const bf16_t* b2 = p.bias2d + (long)((m0 + wm * 128) / p.rows_per_bias2d) * p.N;
#pragma unroll
              for (int q = 0; q < NP; ++q) {
                float t8[8];
                unpack8(*reinterpret_cast<const uint4_*>(b2 + n0 + wn * WC + q * 32 + 8 * fq), t8);
#pragma unroll
                for (int e = 0; e < 8; ++e) bq[q][e] += t8[e];
              }
              if (TAIL) {
                const uint2_ bb = *reinterpret_cast<const uint2_*>(b2 + nt4);
                bt[0] += bf2f(bb[0] & 0xffff); bt[1] += bf2f(bb[0] >> 16);
                bt[2] += bf2f(bb[1] & 0xffff); bt[3] += bf2f(bb[1] >> 16);
              }
            }
            // statistics of the stored output for the next norm (plain epilogue only; host: gemm4_stats_ok).
            // Column (GroupNorm) statistics: the accumulator registers leave no room for per-column sums (the
            // kernel sits at 240-250 VGPRs), so each IG-row-block group of stored values is also written to this
            // wave's slice of LDS buffer 1 (free during the epilogue: the persistent prefetch targets buffer 0, and
            // the next tile restages buffer 1 only after the loop-top barrier) and summed down the rows by lanes
            // owning a column pair: 4 registers per lane.
            constexpr int IG = NJ == 4 ? 4 : 2;
            float* __restrict__ colp = GLU ? nullptr : p.col_part;
            float* __restrict__ rowp = GLU ? nullptr : p.row_part;
            bf16_t* cst = g4_smem + G4_STAGE + wid * (IG * 16 * WC);  // [IG * 16][WC] bf16
            float c0 = 0.f, c1 = 0.f, d0 = 0.f, d1 = 0.f;              // column pair (2 lane, 2 lane + 1)
#pragma unroll
            for (int i0 = 0; i0 < 8; i0 += IG) {
              if constexpr (!GLU) {
                uint4_ rr[IG][NP];
                uint2_ rt[IG];
                if (R) {
#pragma unroll
                  for (int ii = 0; ii < IG; ++ii) {
                    const bf16_t* rrow = R + (long)(m0 + wm * 128 + (i0 + ii) * 16 + fr) * p.ldr + n0 + wn * WC;
#pragma unroll
                    for (int q = 0; q < NP; ++q) rr[ii][q] = *reinterpret_cast<const uint4_*>(rrow + q * 32 + 8 * fq);
                    if (TAIL) rt[ii] = *reinterpret_cast<const uint2_*>(rrow + 2 * NP * 16 + 4 * fq);
                  }
                }
#pragma unroll
                for (int ii = 0; ii < IG; ++ii) {
                  const int i = i0 + ii;
                  bf16_t* crow = C + orow(m0 + wm * 128 + i * 16 + fr) * p.ldc + n0 + wn * WC;
                  // row statistics of this lane's columns, shifted by the row's first stored value in this
                  // slot (lane fq = 0, column 0): (mean, M2) per slot, combined exactly by the finalizer
                  float rs = 0.f, rq = 0.f, rk = 0.f;
#pragma unroll
                  for (int q = 0; q < NP; ++q) {
                    float v[8];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                      v[e] = apply_act<ACT>(acc[i][2 * q][e] * p.alpha + bq[q][e]);
                      v[4 + e] = apply_act<ACT>(acc[i][2 * q + 1][e] * p.alpha + bq[q][4 + e]);
                    }
                    if (R) {
                      float r8[8];
                      unpack8(rr[ii][q], r8);
#pragma unroll
                      for (int e = 0; e < 8; ++e) v[e] += r8[e] * p.res_alpha;
                    }
                    const uint4_ pv = pack8(v);
                    *reinterpret_cast<uint4_*>(crow + q * 32 + 8 * fq) = pv;
                    if (colp) *reinterpret_cast<uint4_*>(cst + (ii * 16 + fr) * WC + q * 32 + 8 * fq) = pv;
                    if (rowp) {  // moments of the stored (bf16-rounded) values: what the consumer reads
                      float f[8];
                      unpack8(pv, f);
                      if (q == 0) rk = __shfl(f[0], fr, 64);
#pragma unroll
                      for (int e = 0; e < 8; ++e) {
                        const float d = f[e] - rk;
                        rs += d;
                        rq = fmaf(d, d, rq);
                      }
                    }
                  }
                  if constexpr (TAIL) {
                    float v[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = apply_act<ACT>(acc[i][NJ - 1][e] * p.alpha + bt[e]);
                    if (R) {
                      v[0] += bf2f(rt[ii][0] & 0xffff) * p.res_alpha; v[1] += bf2f(rt[ii][0] >> 16) * p.res_alpha;
                      v[2] += bf2f(rt[ii][1] & 0xffff) * p.res_alpha; v[3] += bf2f(rt[ii][1] >> 16) * p.res_alpha;
                    }
                    uint2_ o;
                    o[0] = pack2(v[0], v[1]);
                    o[1] = pack2(v[2], v[3]);
                    *reinterpret_cast<uint2_*>(crow + 2 * NP * 16 + 4 * fq) = o;
                    if (colp) *reinterpret_cast<uint2_*>(cst + (ii * 16 + fr) * WC + 2 * NP * 16 + 4 * fq) = o;
                    if (rowp) {
                      const float f[4] = {bf2f(o[0] & 0xffff), bf2f(o[0] >> 16), bf2f(o[1] & 0xffff), bf2f(o[1] >> 16)};
#pragma unroll
                      for (int e = 0; e < 4; ++e) {
                        const float d = f[e] - rk;
                        rs += d;
                        rq = fmaf(d, d, rq);
                      }
                    }
                  }
                  if (rowp) {  // the 4 fq lanes of a row hold its 4 column quarters of this wave's slice
                    rs += __shfl_xor(rs, 16, 64);
                    rq += __shfl_xor(rq, 16, 64);
                    rs += __shfl_xor(rs, 32, 64);
                    rq += __shfl_xor(rq, 32, 64);
                    if (fq == 0) {
                      const long m = m0 + wm * 128 + i * 16 + fr;
                      const int slot = (n0 / BN) * 4 + wn;
                      constexpr float inv_wc = 1.f / WC;  // the slot's column count
                      *reinterpret_cast<float2*>(rowp + (m * p.row_part_slots + slot) * 2) =
                          make_float2(rk + rs * inv_wc, fmaxf(rq - rs * rs * inv_wc, 0.f));
                    }
                  }
                }
                if (colp) {  // one wave's own LDS slice: its ds ops execute in issue order, no barrier needed
                  asm volatile("" ::: "memory");
                  if (lane < WC / 2) {
#pragma unroll 8
                    for (int r = 0; r < IG * 16; ++r) {
                      const uint32_t u = *reinterpret_cast<const uint32_t*>(cst + r * WC + 2 * lane);
                      const float f0 = bf2f(u & 0xffff), f1 = bf2f(u >> 16);
                      c0 += f0;
                      c1 += f1;
                      d0 = fmaf(f0, f0, d0);
                      d1 = fmaf(f1, f1, d1);
                    }
                  }
                  asm volatile("" ::: "memory");
                }
              } else {
                // GLU: (value, gate) column pairs -> the lane's 8 columns give 4 consecutive outputs
                uint2_ rr[IG][NP];
                uint32_t rt[IG];
                if (R) {
#pragma unroll
                  for (int ii = 0; ii < IG; ++ii) {
                    const bf16_t* rrow = R + (long)(m0 + wm * 128 + (i0 + ii) * 16 + fr) * p.ldr + ((n0 + wn * WC) >> 1);
#pragma unroll
                    for (int q = 0; q < NP; ++q) rr[ii][q] = *reinterpret_cast<const uint2_*>(rrow + q * 16 + 4 * fq);
                    if (TAIL) rt[ii] = *reinterpret_cast<const uint32_t*>(rrow + NP * 16 + 2 * fq);
                  }
                }
#pragma unroll
                for (int ii = 0; ii < IG; ++ii) {
                  const int i = i0 + ii;
                  bf16_t* crow = C + (long)(m0 + wm * 128 + i * 16 + fr) * p.ldc + ((n0 + wn * WC) >> 1);
                  uint32_t wq[NP][2];
#pragma unroll
                  for (int q = 0; q < NP; ++q) {
                    float o[4];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                      const int j = 2 * q + h;
                      o[2 * h] = (acc[i][j][0] * p.alpha + bq[q][4 * h]) * apply_act<ACT>(acc[i][j][1] * p.alpha + bq[q][4 * h + 1]);
                      o[2 * h + 1] = (acc[i][j][2] * p.alpha + bq[q][4 * h + 2]) * apply_act<ACT>(acc[i][j][3] * p.alpha + bq[q][4 * h + 3]);
                    }
                    if (R) {
                      o[0] += bf2f(rr[ii][q][0] & 0xffff) * p.res_alpha; o[1] += bf2f(rr[ii][q][0] >> 16) * p.res_alpha;
                      o[2] += bf2f(rr[ii][q][1] & 0xffff) * p.res_alpha; o[3] += bf2f(rr[ii][q][1] >> 16) * p.res_alpha;
                    }
                    wq[q][0] = pack2(o[0], o[1]);
                    wq[q][1] = pack2(o[2], o[3]);
                  }
                  // column groups (2k, 2k + 1): lane quad fq holds outputs 4 fq .. of both; one v_permlane16_swap per
                  // dword gives quads (0, 2) group 2k's and quads (1, 3) group 2k + 1's 8 consecutive outputs -> one
                  // 16-B store per lane instead of two 8-B ones (the GEGLU epilogue is store-issue bound)
#pragma unroll
                  for (int q = 0; q + 1 < NP; q += 2) {
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                      const auto r = __builtin_amdgcn_permlane16_swap(wq[q][e], wq[q + 1][e], false, false);
                      wq[q][e] = r[0];
                      wq[q + 1][e] = r[1];
                    }
                    *reinterpret_cast<uint4_*>(crow + q * 16 + 16 * (fq & 1) + 8 * (fq >> 1)) =
                        uint4_{wq[q][0], wq[q][1], wq[q + 1][0], wq[q + 1][1]};
                  }
                  if constexpr ((NP & 1) != 0) {
                    uint2_ w;
                    w[0] = wq[NP - 1][0];
                    w[1] = wq[NP - 1][1];
                    *reinterpret_cast<uint2_*>(crow + (NP - 1) * 16 + 4 * fq) = w;
                  }
                  if constexpr (TAIL) {
                    float o0 = (acc[i][NJ - 1][0] * p.alpha + bt[0]) * apply_act<ACT>(acc[i][NJ - 1][1] * p.alpha + bt[1]);
                    float o1 = (acc[i][NJ - 1][2] * p.alpha + bt[2]) * apply_act<ACT>(acc[i][NJ - 1][3] * p.alpha + bt[3]);
                    if (R) {
                      o0 += bf2f(rt[ii] & 0xffff) * p.res_alpha;
                      o1 += bf2f(rt[ii] >> 16) * p.res_alpha;
                    }
                    *reinterpret_cast<uint32_t*>(crow + NP * 16 + 2 * fq) = pack2(o0, o1);
                  }
                }
              }
            }
            if (colp && lane < WC / 2)  // column totals over the wave's 128 rows -> partial block (m0 + 128 wm) / 128
              *reinterpret_cast<float4_*>(colp + ((long)((m0 + wm * 128) >> 7) * p.N + n0 + wn * WC + 2 * lane) * 2) =
                  float4_{c0, d0, c1, d1};
            wide_done = true;
            return;
          }
        }
        if (fast && !WIDE) {
          // interior tile: per-column bias hoisted, residual rows prefetched in groups of IG row blocks (all 8
          // at NJ = 4; 2 at NJ = 5, where 160 accumulator registers leave no room for 80 more)
          const bf16_t* __restrict__ bias = p.bias;
          float bj[NJ][4];
    #pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int n = n0 + wn * WC + j * 16 + 4 * fq;
            if (bias) {
              const uint2_ bb = *reinterpret_cast<const uint2_*>(bias + n);
              bj[j][0] = bf2f(bb[0] & 0xffff); bj[j][1] = bf2f(bb[0] >> 16);
              bj[j][2] = bf2f(bb[1] & 0xffff); bj[j][3] = bf2f(bb[1] >> 16);
            } else {
              bj[j][0] = bj[j][1] = bj[j][2] = bj[j][3] = 0.f;
            }
          }
          constexpr int IG = NJ == 4 ? 8 : 2;
          if constexpr (!GLU) {
    #pragma unroll
            for (int i0 = 0; i0 < 8; i0 += IG) {
              uint2_ rr[IG][NJ];
              if (R) {
    #pragma unroll
                for (int ii = 0; ii < IG; ++ii)
    #pragma unroll
                  for (int j = 0; j < NJ; ++j)
                    rr[ii][j] = *reinterpret_cast<const uint2_*>(R + (long)(m0 + wm * 128 + (i0 + ii) * 16 + fr) * p.ldr +
                                                                 n0 + wn * WC + j * 16 + 4 * fq);
              }
    #pragma unroll
              for (int ii = 0; ii < IG; ++ii) {
                const int i = i0 + ii;
                const int m = m0 + wm * 128 + i * 16 + fr;
    #pragma unroll
                for (int j = 0; j < NJ; ++j) {
                  const int n = n0 + wn * WC + j * 16 + 4 * fq;
                  float v[4];
    #pragma unroll
                  for (int e = 0; e < 4; ++e) v[e] = apply_act<ACT>(acc[i][j][e] * p.alpha + bj[j][e]);
                  if (R) {
                    v[0] += bf2f(rr[ii][j][0] & 0xffff) * p.res_alpha; v[1] += bf2f(rr[ii][j][0] >> 16) * p.res_alpha;
                    v[2] += bf2f(rr[ii][j][1] & 0xffff) * p.res_alpha; v[3] += bf2f(rr[ii][j][1] >> 16) * p.res_alpha;
                  }
                  uint2_ o;
                  o[0] = pack2(v[0], v[1]);
                  o[1] = pack2(v[2], v[3]);
                  *reinterpret_cast<uint2_*>(C + orow(m) * p.ldc + n) = o;
                }
              }
            }
          } else {
    #pragma unroll
            for (int i0 = 0; i0 < 8; i0 += IG) {
              uint32_t rr[IG][NJ];
              if (R) {
    #pragma unroll
                for (int ii = 0; ii < IG; ++ii)
    #pragma unroll
                  for (int j = 0; j < NJ; ++j)
                    rr[ii][j] = *reinterpret_cast<const uint32_t*>(R + (long)(m0 + wm * 128 + (i0 + ii) * 16 + fr) * p.ldr +
                                                                  ((n0 + wn * WC + j * 16 + 4 * fq) >> 1));
              }
    #pragma unroll
              for (int ii = 0; ii < IG; ++ii) {
                const int i = i0 + ii;
                const int m = m0 + wm * 128 + i * 16 + fr;
    #pragma unroll
                for (int j = 0; j < NJ; ++j) {
                  const int nc = (n0 + wn * WC + j * 16 + 4 * fq) >> 1;
                  float o0 = (acc[i][j][0] * p.alpha + bj[j][0]) * apply_act<ACT>(acc[i][j][1] * p.alpha + bj[j][1]);
                  float o1 = (acc[i][j][2] * p.alpha + bj[j][2]) * apply_act<ACT>(acc[i][j][3] * p.alpha + bj[j][3]);
                  if (R) {
                    o0 += bf2f(rr[ii][j] & 0xffff) * p.res_alpha;
                    o1 += bf2f(rr[ii][j] >> 16) * p.res_alpha;
                  }
                  *reinterpret_cast<uint32_t*>(C + (long)m * p.ldc + nc) = pack2(o0, o1);
                }
              }
            }
          }
          return;
        }
    #pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int m = m0 + wm * 128 + i * 16 + fr;
          if (m >= p.M) continue;
    #pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int n = n0 + wn * WC + g4_col<BN, WIDE>(j, fq);
            if (n >= p.N) continue;
            float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
            epilogue4<GLU, ACT>(p, CONV == 3 ? C + (orow(m) - m) * p.ldc : C, R, m, n, v, b);
          }
        }
      }
    };
    epilogue(em0, en0);
    if (!more) break;
    setup();  // the next tile's offsets again (dead across the epilogue, so they cost no registers there)
  }
}

// ---------------------------------------------------------------------------- host side
bool gemm4_supported(const GemmArgs& a) {
  if (a.in_scale != nullptr) return false;
  if (a.K % 8 != 0 || a.lda % 8 != 0 || a.ldw % 8 != 0) return false;  // 16-B source chunks
  // weight slices: whole 256-row tiles per slice, plain batch-1 GEMM
  if (a.w_slice_rows != 0 && (a.w_slice_rows % G4_BM != 0 || a.conv || a.batch > 1 || a.M % a.w_slice_rows != 0))
    return false;
  if (a.conv) {
    if (a.Cin % 64 != 0) return false;
    if (a.A2 != nullptr && a.Cin1 % 64 != 0) return false;
    if (a.upsample == 2) {  // phase conv: one image and phase per tile, output rows remapped (no residual / row stats)
      if (a.KH != 2 || a.KW != 2 || a.OH != 2 * a.H || a.OW != 2 * a.Wd) return false;
      if ((a.H & (a.H - 1)) != 0 || (a.Wd & (a.Wd - 1)) != 0) return false;  // rows map by shifts (up2_row)
      const int hw = a.H * a.Wd;  // below 256: 256 / hw images per group (whole groups, no per-image bias)
      if (hw < G4_BM && (a.Nimg % (G4_BM / hw) != 0 || a.bias2d != nullptr)) return false;
      if (a.residual != nullptr || a.row_part != nullptr || a.row_mr != nullptr || a.gate != nullptr) return false;
      if (a.batch > 1 || a.glu) return false;
    }
  }
  return true;
}

bool gemm4_stats_ok(const GemmArgs& a, int bn) {
  const auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!gemm4_supported(a) || a.glu || a.gate != nullptr || (a.batch > 1)) return false;
  if (a.M % G4_BM != 0 || a.N % bn != 0 || a.ldc % 8 != 0 || !al16(a.C)) return false;
  if (a.residual != nullptr && (a.ldr % 8 != 0 || !al16(a.residual))) return false;
  if (a.bias != nullptr && !al16(a.bias)) return false;
  if (a.bias2d != nullptr && (a.rows_per_bias2d % 128 != 0 || a.N % 8 != 0 || !al16(a.bias2d))) return false;
  // phase conv over image groups (H W < 256): the GEMM's 128-row blocks interleave the group's images, and the partials'
  // consumer maps block b to image b * 128 / (OH OW) -- statistics from a pass over the output instead
  if (a.upsample == 2 && a.H * a.Wd < G4_BM) return false;
  return true;
}

// persistent grid width: the CU count rounded down to a multiple of 8 (one workgroup per CU; every tile
// of a workgroup stays on its XCD)
static int g4_persist_width() {
  static int w = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 8)
      cus = 256;
    return cus & ~7;
  }();
  return w;
}

template <int CONV, bool GLU, int ACT, int VAR = 4>
static void g4_launch(const GemmArgs& a, float* ws, int splits, int kps, int bn, hipStream_t s) {
  dim3 grid(1, splits > 1 ? splits : (a.batch > 0 ? a.batch : 1));
  const auto width = [&](long tiles) {  // persistent: at most one workgroup per CU, tiles walked in a loop
    return (unsigned)((VAR & 8) && splits <= 1 ? std::min<long>(tiles, g4_persist_width()) : tiles);
  };
  if (bn == 320) {
    grid.x = width(((a.M + G4_BM - 1) / G4_BM) * ((a.N + 319) / 320));
    const size_t lds = (size_t)2 * G4T<320>::STAGE * sizeof(bf16_t);
    if (splits > 1) gemm4_kernel<CONV, GLU, ACT, true, VAR, 320><<<grid, 512, lds, s>>>(a, ws, kps);
    else gemm4_kernel<CONV, GLU, ACT, false, VAR, 320><<<grid, 512, lds, s>>>(a, ws, kps);
  } else {
    grid.x = width(((a.M + G4_BM - 1) / G4_BM) * ((a.N + 255) / 256));
    const size_t lds = (size_t)2 * G4T<256>::STAGE * sizeof(bf16_t);
    if (splits > 1) gemm4_kernel<CONV, GLU, ACT, true, VAR, 256><<<grid, 512, lds, s>>>(a, ws, kps);
    else gemm4_kernel<CONV, GLU, ACT, false, VAR, 256><<<grid, 512, lds, s>>>(a, ws, kps);
  }
}

// splits > 1 requires ws ([splits][M][N] fp32); the split-K fold + epilogue runs afterwards.
template <int VAR>
static void g4_dispatch(const GemmArgs& a, float* ws, int splits, int kps, int bn, hipStream_t s);

void launch_gemm4(const GemmArgs& a, float* ws, int splits, int bn, hipStream_t s, bool persist) {
  if (ws == nullptr) splits = 1;  // (phase conv: the fold maps GEMM rows to output pixels, up2_out_row)
  const long kt = (a.K + G4_BK - 1) / G4_BK;
  const int kps = (int)(((kt + splits - 1) / splits) * G4_BK);
  // wide epilogue (VAR bit 4) in production: +1-3 % on K >= 2048, +14-24 % on the K = 320 SD2.1 GEMMs
  // (tools/gemm_lab, profiles/gemm_wide_epilogue_round3.md)
  // persistent: + VAR bit 5 (the epilogue's stores stay in flight into the next tile; lab +0-4 %)
  if (persist && splits <= 1) g4_dispatch<60>(a, ws, splits, kps, bn, s);
  else g4_dispatch<20>(a, ws, splits, kps, bn, s);
  if (splits > 1) launch_splitk_epilogue(a, ws, splits, s);
}

template <int VAR>
static void g4_dispatch(const GemmArgs& a, float* ws, int splits, int kps, int bn, hipStream_t s) {
  if (a.conv) {
    if (a.upsample == 2) {
      if (a.act == ACT_SILU) g4_launch<3, false, ACT_SILU, VAR>(a, ws, splits, kps, bn, s);
      else g4_launch<3, false, ACT_NONE, VAR>(a, ws, splits, kps, bn, s);
    } else if (a.upsample) {
      if (a.act == ACT_SILU) g4_launch<2, false, ACT_SILU, VAR>(a, ws, splits, kps, bn, s);
      else g4_launch<2, false, ACT_NONE, VAR>(a, ws, splits, kps, bn, s);
    } else {
      if (a.act == ACT_SILU) g4_launch<1, false, ACT_SILU, VAR>(a, ws, splits, kps, bn, s);
      else g4_launch<1, false, ACT_NONE, VAR>(a, ws, splits, kps, bn, s);
    }
  } else if (a.glu) {
    if (a.act == ACT_SILU) g4_launch<0, true, ACT_SILU, VAR>(a, ws, splits, kps, bn, s);
    else if (a.act == ACT_GELU_TANH) g4_launch<0, true, ACT_GELU_TANH, VAR>(a, ws, splits, kps, bn, s);
    else g4_launch<0, true, ACT_GELU, VAR>(a, ws, splits, kps, bn, s);
  } else {
    switch (a.act) {
      case ACT_SILU: g4_launch<0, false, ACT_SILU, VAR>(a, ws, splits, kps, bn, s); break;
      case ACT_GELU: g4_launch<0, false, ACT_GELU, VAR>(a, ws, splits, kps, bn, s); break;
      case ACT_GELU_TANH: g4_launch<0, false, ACT_GELU_TANH, VAR>(a, ws, splits, kps, bn, s); break;
      case ACT_QUICK_GELU: g4_launch<0, false, ACT_QUICK_GELU, VAR>(a, ws, splits, kps, bn, s); break;
      case ACT_RELU: g4_launch<0, false, ACT_RELU, VAR>(a, ws, splits, kps, bn, s); break;
      default: g4_launch<0, false, ACT_NONE, VAR>(a, ws, splits, kps, bn, s); break;
    }
  }
}

#ifdef SHAI_GEMM_LAB
// Lab entry (tools/gemm_lab, built with -DSHAI_GEMM_LAB only): schedule variant `var` (see G4Sched) with the
// full epilogue dispatch (conv / GLU / activations), no split-K.
void launch_gemm4_var(const GemmArgs& a, int var, int bn, hipStream_t s) {
  const int kps = (int)(((a.K + G4_BK - 1) / G4_BK) * G4_BK);
  switch (var) {
    case 20: g4_dispatch<20>(a, nullptr, 1, kps, bn, s); break;
    case 60: g4_dispatch<60>(a, nullptr, 1, kps, bn, s); break;
    default: break;
  }
}
#endif

}  // namespace shai
