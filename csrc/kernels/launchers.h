// Host-side launcher interface of the HIP kernels.  Kernel translation units
// include only this header and <hip/hip_runtime.h> (no torch headers), which
// keeps their hipcc compile fast; csrc/bindings.cpp adapts torch tensors.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace shai {
typedef uint16_t bf16_t;

// ---------------------------------------------------------------- norms
struct RowNormArgs {
  const bf16_t* x;
  const bf16_t* residual;   // optional: x + residual is normalised
  const bf16_t* w;          // optional weight [D]
  const bf16_t* b;          // optional bias [D] (LayerNorm only)
  bf16_t* out;
  bf16_t* residual_out;     // optional: receives x + residual
  int rows, D;
  long x_stride, out_stride;  // row strides in elements
  float eps;
  float w_offset;           // y = norm(x) * (w + w_offset) + b
  int rows_per_w;           // >0: w/b advance by w_stride every rows_per_w rows (AdaLN modulation per image)
  long w_stride;
};
void launch_rmsnorm(const RowNormArgs& a, hipStream_t s);
void launch_layernorm(const RowNormArgs& a, hipStream_t s);

struct GroupNormArgs {
  const bf16_t* x;   // [N, HW, C] channels-last
  const bf16_t* gamma;
  const bf16_t* beta;
  float* partials;   // [N, 256, G, 2] workspace
  float* scale;      // [N, C]
  float* shift;      // [N, C]
  bf16_t* out;       // apply output (optional)
  int N, HW, C, G;
  float eps;
  int silu;
  const bf16_t* x2;  // optional second source: channels [C1, C) (fused concat; x then holds [0, C1))
  int C1;
  unsigned* counters;  // optional [N] zeroed tickets: finalize fused into the stats launch
};
int gn_num_blocks(int N, int HW, int C);
void launch_groupnorm_stats(const GroupNormArgs& a, hipStream_t s);
void launch_groupnorm_apply(const GroupNormArgs& a, hipStream_t s);
// Norm statistics produced by a GEMM epilogue (GemmArgs::col_part / row_part) and their fallback passes:
//   col partials [M / 128, N, 2] (sum, sum of squares per 128-row block and column) of x [M, N] (row stride ldx)
void launch_col_partials(const bf16_t* x, long M, int N, long ldx, float* part, hipStream_t s);

//   GroupNorm (scale, shift) [Nimg, C1 + C2] from the col partials of x (C1 channels) and optional x2 (C2)
void launch_gn_from_partials(const float* part1, int C1, const float* part2, int C2, int Nimg, int HW, int G,
                             const bf16_t* gamma, const bf16_t* beta, float eps, float* scale, float* shift,
                             hipStream_t s);
//   LayerNorm row moments mr [M, 2] = (mean, rstd) from row partials [M, slots, 2], or directly from x
void launch_row_moments_from_partials(const float* part, long M, int slots, int N, float eps, float* mr,
                                      hipStream_t s);
void launch_row_moments(const bf16_t* x, long M, int N, long ldx, float eps, float* mr, hipStream_t s);

// ---------------------------------------------------------------- elementwise
void launch_cache_flush(const void* buf, size_t bytes, unsigned* sink, hipStream_t s);
// out[t, i] = act(x[t, i]) * x[t, F + i]   (gated MLP, unfused fallback), F = D/2
void launch_gated_act(const bf16_t* x, bf16_t* out, long rows, int F, long x_stride, int act, int gate_first,
                      hipStream_t s);
// out = act(x * alpha + bias) (+ residual)  over [rows, D]
void launch_bias_act(const bf16_t* x, const bf16_t* bias, const bf16_t* residual, bf16_t* out, long rows, int D,
                     int act, float alpha, hipStream_t s);
// Rotary embedding in-place on q/k heads: x [T, H, Dh] (token stride given),
// cos/sin tables [max_pos, rot_dim/2] fp32, positions [T] int32.
void launch_rope(bf16_t* x, const int* positions, const float* cos, const float* sin, int T, int H, int Dh,
                 int rot_dim, long tok_stride, int neox, hipStream_t s);
// Flux 3-axis rope with precomputed per-token (cos, sin) pairs [T, Dh/2].
// Flux: in-place per-head RMSNorm of q and k (weights optional) + pair RoPE (cos/sin optional, [S, D/2]).
// x: [rows, >= 2*H*D] with row stride ld; q at column 0, k at column H*D; row r uses rope position r % S.
void launch_qk_norm_rope(bf16_t* x, long ld, int rows, int S, int H, int D, const bf16_t* qw, const bf16_t* kw,
                         const float* cs, const float* sn, float eps, hipStream_t s);
// Llama/Mistral: NeoX RoPE on q (in place) and k + paged KV-cache write of k, v from the packed QKV rows.
void launch_rope_qkv_cache(bf16_t* qkv, long ld, const int* pos, const float* cos, const float* sin, bf16_t* k_cache,
                           bf16_t* v_cache, const int* slots, int T, int H, int Hkv, int D, hipStream_t s);
void launch_rope_pairs(bf16_t* x, const float* cos, const float* sin, int B, int T, int H, int Dh, long batch_stride,
                       long tok_stride, hipStream_t s);
// Scheduler step fused with classifier-free guidance (all fp32 math):
//   eps = eu + g * (ec - eu)  (model_out holds [uncond; cond] halves when cfg)
//   DDIM (eta=0):  x0 = (x - sqrt(1-a) eps)/sqrt(a) ; x' = sqrt(ap) x0 + sqrt(1-ap) eps
//   v-prediction variants handled by pred_type (0 eps, 1 v, 2 flow (x' = x + dt * v))
void launch_sched_step_rows(const bf16_t* mo, bf16_t* lat, long n, long per_row, int cfg, float g, int pred,
                            const float* rows, hipStream_t s);
void launch_sched_step(const bf16_t* model_out, bf16_t* latents, long n, int cfg, float guidance, int pred_type,
                       float a_t, float a_prev, float dt, hipStream_t s);
// Row softmax in-place (fp32 math), bf16 rows of length D
void launch_softmax(bf16_t* x, long rows, int D, float scale, hipStream_t s);
// Embedding gather: out[t] = table[ids[t]]
void launch_embedding(const int* ids, const bf16_t* table, bf16_t* out, long T, int D, hipStream_t s);
void launch_token_feedback(int* ids, const int* rowmap, const int* prev, int n, hipStream_t s);

// ---------------------------------------------------------------- GEMM / conv
struct GemmArgs {
  // C[b, m, n] = act(alpha * sum_k A[b, m, k] * W[b, n, k] + bias[n] + bias2d[m/rows_per_bias2d, n]) + residual[b, m, n]
  const bf16_t* A;
  const bf16_t* W;
  bf16_t* C;
  const bf16_t* bias;      // [N] optional
  const bf16_t* bias2d;    // [M / rows_per_bias2d, N] optional (e.g. time-embedding per image)
  const bf16_t* residual;  // [M, N] optional (same layout as C)
  int M, N, K;
  long lda, ldw, ldc, ldr;  // row strides (elements)
  long batch_a, batch_w, batch_c, batch_r;  // batch strides (elements)
  int batch;
  int rows_per_bias2d;
  float alpha;
  float res_alpha;          // C = epi + res_alpha * residual
  int act;                  // Act enum
  int glu;                  // 1: gated output, weights interleaved (a,g) pairs -> C has N/2 cols: act(g) * a
  // implicit-GEMM convolution (A is an NHWC activation, K = KH*KW*Cin)
  int conv;                 // 0 = plain GEMM
  int Nimg, H, Wd, Cin, OH, OW, KH, KW, stride, pad, upsample;  // upsample: nearest-2x fused into gather
  const bf16_t* A2;         // optional second source: channels [Cin1, Cin) come from A2 (fused concat)
  int Cin1;
  // fused GroupNorm apply on the gathered A operand: a = act(x * scale[n,c] + shift[n,c])
  const float* in_scale;
  const float* in_shift;
  int in_act;
  // AdaLN-Zero gate: out = gate[(b*M + m) / rows_per_gate, n] * epi(...) + residual (v2 kernel only)
  const bf16_t* gate;
  long gate_stride;
  int rows_per_gate;
  // RMSNorm folded into the GEMM (skinny kernel / split-K fold only): C = rstd[m] * (A W^T) ... with
  // rstd[m] = rsqrt(mean_k A[m, k]^2 + rms_eps); the norm gain is pre-multiplied into W's columns.
  int rms;
  float rms_eps;
  // fp8 weights (skinny kernel only): W is e4m3 [N, K] bytes, w_scale[n] fp32 per output row
  const float* w_scale;
  int w_nt;                 // skinny kernel: weight stream with the nt cache policy (set by its launcher)
  // LayerNorm folded into the GEMM (v4 kernel, unsplit, batch 1): acc <- rstd[m] * (acc - mean[m] * col_s[n])
  // before the epilogue; the norm gain is pre-multiplied into W's columns and its shift into the bias
  const float* row_mr;      // [M, 2] (mean, rstd) of the un-normalised A rows
  const float* col_s;       // [N] column sums of the gain-folded W (fp32, from its bf16 values)
  // output statistics for the NEXT norm, written by the v4 wide epilogue (gemm4_stats_ok); other kernels leave
  // them to the fallback passes of launch_out_stats
  float* col_part;          // [M / 128, N, 2]: per 128-row block and column (sum, sum of squares) -> GroupNorm
  float* row_part;          // [M, row_part_slots, 2]: per row and slot (mean, M2) of that slot's columns, shifted
  int row_part_slots;       //   by the row's first value -> LayerNorm (Chan's combine in row_moments_part_kernel
                            //   assumes equal column counts: every slot covers N / slots columns);
                            //   slots = 4 * column tiles
  // > 0: rows [s w_slice_rows, (s + 1) w_slice_rows) multiply weight slice s (W is [M / w_slice_rows][N][ldw]; v4
  // kernel only, w_slice_rows % 256 == 0): a per-image weight, e.g. a GroupNorm's per-image scale folded into W
  int w_slice_rows;
};
// (conv, GLU, activation) epilogue variants the tile kernels (v2 / v4 / four-wave / W-stationary / halo conv)
// instantiate: convolutions NONE / SILU, GLU SILU / GELU / GELU_TANH, plain GEMMs every activation.  Any other
// combination is rejected by every tile config (gemm2_cfg_supported), never run as a neighbouring variant.
inline bool tile_act_supported(const GemmArgs& a) {
  if (a.conv) return !a.glu && (a.act == 0 || a.act == 1);       // ACT_NONE, ACT_SILU
  if (a.glu) return a.act == 1 || a.act == 2 || a.act == 3;      // ACT_SILU, ACT_GELU, ACT_GELU_TANH
  return true;
}
void launch_dequant_fp8_rows(const uint8_t* w8, const float* scale, bf16_t* out, long N, int K, hipStream_t s);
// fp8 e4m3 MFMA GEMM (gemm_f8.hip): C = epi(a_scale[m] w_scale[n] A8 W8^T); A8 / W8 are e4m3 bytes, lda / ldw in
// bytes; cfg 0 = 256 x 128 tile, 1 = 128 x 128
bool gemm_f8_supported(const GemmArgs& a);
void launch_gemm_f8(const GemmArgs& a, const uint8_t* A8, const uint8_t* W8, const float* a_scale,
                    const float* w_scale, int cfg, hipStream_t s);
// per-row e4m3 quantisation of a bf16 activation (scale = absmax / 448, times the row's RMSNorm rstd when
// rms_eps >= 0)
bool quant_rows_fp8_supported(int K);
void launch_quant_rows_fp8(const bf16_t* x, long ldx, int M, int K, uint8_t* out, long ldo, float* scale,
                           float rms_eps, hipStream_t s);
void launch_gemm(const GemmArgs& a, hipStream_t s);       // v1: register-staged (supports fused GN gather)
// v2: LDS-DMA staged, tile configs + split-K (ws: fp32 workspace of gemm2_workspace_bytes, may be null)
void launch_gemm2(const GemmArgs& a, float* ws, hipStream_t s);
size_t gemm2_workspace_bytes(const GemmArgs& a);
void gemm2_plan(const GemmArgs& a, int* cfg, int* splits);
void launch_gemm2_cfg(const GemmArgs& a, float* ws, int cfg, int splits, hipStream_t s);
int gemm2_num_cfgs();
bool gemm2_cfg_supported(const GemmArgs& a, int cfg);
bool gemm2_cfg_splittable(int cfg);  // false: the config always runs the whole K (split-K choices are moot)
// v5: four-wave GEMM / implicit-GEMM conv (gemm_w4.hip), bn = 256: 256 x 256 tiles, bn = 320: 192 x 320 tiles
bool gemm_w4_supported(const GemmArgs& a);
void launch_gemm_w4(const GemmArgs& a, int bn, hipStream_t s);
// v6: W-stationary low-K GEMM (gemm_ws.hip): K = 320, N % 320 == 0, persistent over M, weights in VGPRs
bool gemm_ws_supported(const GemmArgs& a);
void launch_gemm_ws(const GemmArgs& a, hipStream_t s);
// the same with the next LayerNorm in the epilogue: C = x W^T + bias + res_alpha R and C2 = LayerNorm(C) gamma + beta
// (N = 320: the whole row in one workgroup; residual, no activation)
bool gemm_ws_lnout_supported(const GemmArgs& a);
void launch_gemm_ws_lnout(const GemmArgs& a, bf16_t* C2, const bf16_t* gamma, const bf16_t* beta, float eps,
                          hipStream_t s);
// halo-tiled 3x3 conv (conv_halo.hip): stride 1 / pad 1, OW in {16, 32, 64}, Cin (and the concat split) multiples of
// 64, N % 160 or N % 128 == 0; the input's GroupNorm + SiLU (in_scale / in_shift, one [2, N, Cin] allocation) applied
// once per staged element in LDS; writes col_part (GroupNorm partials of the output) when set.  waves: 4 or 8 (0:
// SHAI_HALO_WAVES, default 8)
bool conv_halo_supported(const GemmArgs& a);
void launch_conv_halo(const GemmArgs& a, hipStream_t s, int waves);
// whether config cfg is raced by the autotuner (retired configs still run a cached choice, on their successor)
bool gemm2_cfg_candidate(int cfg);
void launch_splitk_epilogue(const GemmArgs& a, const float* ws, int splits, hipStream_t s);
// v4: 8-phase ping-pong 256x256 / 256x320 LDS-DMA GEMM / conv (gemm_8ph.hip); config indices
// gemm2_num_cfgs() - 2 (bn 256) and - 1 (bn 320)
bool gemm4_supported(const GemmArgs& a);
// every tile of this problem takes the v4 wide epilogue (the only path that writes col_part / row_part)
bool gemm4_stats_ok(const GemmArgs& a, int bn);
void launch_gemm4(const GemmArgs& a, float* ws, int splits, int bn, hipStream_t s, bool persist = false);
// skinny (decode-shaped, M <= 64) streaming GEMM; ws: skinny_workspace_bytes (fp32 split-K partials)
bool skinny_supported(const GemmArgs& a);
int skinny_kgroups(const GemmArgs& a);        // heuristic K-group count
int skinny_max_kgroups(const GemmArgs& a);    // largest K-group count worth trying (autotuner)
size_t skinny_workspace_bytes(const GemmArgs& a);
size_t skinny_workspace_bytes_kg(const GemmArgs& a, int kg);
void launch_skinny(const GemmArgs& a, float* ws, hipStream_t s);
// fold = false (kg > 1, no fixup): leave the fp32 partials in ws for a consumer kernel (no fold launch)
void launch_skinny_kg(const GemmArgs& a, float* ws, int kg, hipStream_t s, bool fixup = false, bool fold = true);
// this launch's slice of the in-kernel split-K arrival tickets (nullptr: none available -> no fixup)
unsigned* skinny_ticket_slice(hipStream_t s, int ntiles);
// skinny2 (gemv2.hip): 128-row W tiles, whole K-step per wave, M <= 64, bf16 weights; split-K always fixed up
// in the launch (ws of skinny2_workspace_bytes)
bool skinny2_supported(const GemmArgs& a);
int skinny2_max_kgroups(const GemmArgs& a);
size_t skinny2_workspace_bytes(const GemmArgs& a, int kg);
void launch_skinny2(const GemmArgs& a, float* ws, int kg, bool deep, hipStream_t s);
void gemm2_cfg_info(int cfg, int* bm, int* bn);

// ---------------------------------------------------------------- attention
struct AttnArgs {
  const bf16_t* q;  // [B, Sq, Hq, D] with strides
  const bf16_t* k;  // [B, Skv, Hkv, D]
  const bf16_t* v;
  bf16_t* o;        // [B, Sq, Hq, D] with strides
  int B, Sq, Skv, Hq, Hkv, D;
  long q_bs, q_ts, k_bs, k_ts, v_bs, v_ts, o_bs, o_ts;  // batch / token strides (elements); head stride = D
  float scale;
  int causal;
  int causal_offset;        // query i sees keys <= i + causal_offset
  const int* kv_lens;       // optional [B] valid key count per batch
  const int* q_lens;        // optional [B] valid query count; causal offset becomes kv_len - q_len
  const int* q_start;       // optional [B] packed varlen: sequence b's queries / outputs are rows
                            // q_start[b] .. q_start[b] + q_lens[b] - 1 of a flat [T, Hq, D] q / o (q_bs unused)
  const bf16_t* bias;       // optional additive bias [Hq, Sq, Skv] (bf16), broadcast over batch
  // paged K/V (LLM prefill over cached context): block tables of 64-token blocks
  const int* block_table;   // optional [B, max_blocks]
  int max_blocks;
  long kc_bs, kc_hs;        // cache strides: block stride, head stride (elements); token stride = D
};
void launch_flash_attn(const AttnArgs& a, hipStream_t s);
// v2 (attention2.hip): 8-wave ping-pong, LDS-DMA K/V ring; launch_flash_attn dispatches to it when supported
bool flash2_supported(const AttnArgs& a);
bool flash64_supported(const AttnArgs& a);
void launch_flash64(const AttnArgs& a, hipStream_t s);
void launch_flash2(const AttnArgs& a, hipStream_t s);
// flash64 with LDS-DMA K/V staging (attention3.hip; launch_flash64 routes to it, SHAI_FLASH64_DMA=0 opts out)
bool flash64_dma_supported(const AttnArgs& a);
void launch_flash64_dma(const AttnArgs& a, hipStream_t s);
// the same pipeline with two 32-query groups per wave (256 queries per workgroup, flash64_dma_supported contract;
// launch_flash64 picks it for grids of >= 1024 such workgroups)
void launch_flash64_x2(const AttnArgs& a, hipStream_t s);
// D = 128 with two 32-query groups per wave (attention3.hip; 256 queries per workgroup, one workgroup per CU): Flux
// joint attention / LLM prefill; opt-in over flash2 for D = 128 (SHAI_FLASH128X2=1 / set_flash128x2: measured slower)
bool flash128x2_supported(const AttnArgs& a);
void launch_flash128x2(const AttnArgs& a, hipStream_t s);
int flash128x2_mode();
int set_flash128x2(int mode);   // -1 keeps the mode; returns the previous one
// D = 512 single-head fused attention (attention3.hip; the VAE mid-block)
bool attn512_supported(const AttnArgs& a);
void launch_attn512(const AttnArgs& a, hipStream_t s);

struct DecodeAttnArgs {
  const bf16_t* q;          // [B, Hq, D]
  const bf16_t* k_cache;    // [num_blocks, Hkv, 64, D]
  const bf16_t* v_cache;
  bf16_t* o;                // [B, Hq, D]
  const int* block_table;   // [B, max_blocks]
  const int* ctx_lens;      // [B]
  float* ws;                // split-K workspace
  int B, Hq, Hkv, D, max_blocks, num_splits;
  long q_bs, o_bs;
  float scale;
  // fused decode step (knew != nullptr): q is un-roped; this step's k / v rows ([B, Hkv, D] at row stride
  // new_bs) are roped / taken from here, written into the cache at slots[b] (-1: padding row) and attended
  // from registers; ctx_lens count the new token, the cache holds ctx_lens - 1 of them
  const bf16_t* knew;
  const bf16_t* vnew;
  long new_bs;
  const int* positions;
  const float* rope_cos;    // [max_pos, D / 2] NeoX halves
  const float* rope_sin;
  const int* slots;
  // QKV GEMM fold fused in (qkv_ws != nullptr): q / k / v are read as the sum of qkv_kg fp32 split-K partial slabs
  // [kg][B][qkv_n] of the skinny kernel, times the folded-RMSNorm row scale from the [kg][B] row sums of squares
  // (qkv_k = the GEMM's K, qkv_eps its epsilon), rounded to bf16 -- what the separate fold would have stored
  const float* qkv_ws;
  int qkv_kg, qkv_n, qkv_k;
  float qkv_eps;
};
void launch_decode_attn(const DecodeAttnArgs& a, hipStream_t s);
// short-context decode routing (D 128, GQA 4, one split -> the wave-per-block kernel); SHAI_DECODE_WB=0 / mode 0: split kernel
int decode_wb_mode();
int set_decode_wb(int mode);   // -1 keeps the mode; returns the previous one
size_t decode_attn_workspace(int B, int Hq, int D, int num_splits);

// Write new K/V tokens into the paged cache.
void launch_kv_write(const bf16_t* k, const bf16_t* v, bf16_t* k_cache, bf16_t* v_cache, const int* slot_mapping,
                     int T, int Hkv, int D, long k_ts, long v_ts, hipStream_t s);

// ---------------------------------------------------------------- sampling
// Per-row temperature / top-k (<= 1024 candidates) / top-p sampling from bf16 or fp32 logits [B, ld].
void launch_sample(const void* logits, bool bf16, long ld, int B, int V, const float* temps, const int* top_k,
                   const float* top_p, const float* uniforms, int* out, hipStream_t s);
}  // namespace shai
