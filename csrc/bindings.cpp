// torch operator registrations (namespace `shai`) for the gfx950 HIP kernels.
// Every op writes into caller-allocated outputs on the current HIP stream and
// never allocates or synchronises, so the ops are hipGraph-capturable.
// Shape/stride/alignment preconditions the kernels rely on are checked here,
// on the host, before launch (a bad launch on the box can reset the node).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <unordered_map>
#include <algorithm>
#include <vector>

#include "kernels/launchers.h"

using at::Tensor;
using c10::optional;

namespace {

#define SHAI_CHECK(cond, ...) TORCH_CHECK(cond, "shai: ", __VA_ARGS__)

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

// Halo-tiled conv routing (conv_halo.hip): 0 off (default), 1 GroupNorm-fused convs, 2 also plain 3x3 convs;
// SHAI_HALO_CONV sets it, the set_halo_conv op changes it at run time (A/B in one process).  g_halo_waves: 0 = the
// kernel's default wave layout (SHAI_HALO_WAVES), 4 / 8 pin one.  Off by default: at the SD2.1 batch-32 shapes the
// in-LDS normalisation costs more than the apply pass it replaces (profiles/halo_conv_round6.md: e.g. 64x64x320
// 561 us fused vs 497 us apply + tuned conv), so a norm= conv runs the apply pass + the tuned conv.
int g_halo_mode = -1;
int g_halo_waves = 0;
int halo_conv_mode() {
  if (g_halo_mode < 0) {
    const char* e = getenv("SHAI_HALO_CONV");
    g_halo_mode = e ? atoi(e) : 0;
  }
  return g_halo_mode;
}
int64_t set_halo_conv(int64_t mode, int64_t waves) {
  const int prev = halo_conv_mode();
  if (mode >= 0) g_halo_mode = (int)mode;
  if (waves >= 0) g_halo_waves = (int)waves;
  return prev;
}

// v2 GEMM (LDS-DMA) unless the problem needs v1 features (fused GN gather) or
// exceeds the 2 GiB buffer-descriptor range.  SHAI_GEMM_V1=1 forces v1.
bool use_v2(const shai::GemmArgs& g, long a_bytes, long w_bytes, long a2_bytes) {
  static const bool force_v1 = getenv("SHAI_GEMM_V1") != nullptr;
  if (force_v1 || g.in_scale != nullptr) return false;
  const long lim = 0x7fffffffL - 64;
  if (a_bytes > lim || w_bytes > lim || a2_bytes > lim) return false;
  for (int c = 0; c < shai::gemm2_num_cfgs(); ++c)
    if (shai::gemm2_cfg_supported(g, c)) return true;
  return false;
}

// ---- GEMM autotuner: the first eager call of a problem shape times every
// (tile config, split-K) candidate with HIP events and caches the winner.
// Calls made while the stream is being captured into a graph (or with
// SHAI_GEMM_AUTOTUNE=0) use the cached choice, else the analytic planner.
struct Choice {
  int cfg, splits;
};
std::mutex g_tune_mu;
std::unordered_map<std::string, Choice> g_tuned;

bool lib_supported(const shai::GemmArgs& g) {
  return g.conv == 0 && !g.row_mr && g.batch <= 1 && !g.w_slice_rows && !g.glu && g.act == 0 && !g.bias2d && !g.gate &&
         !g.rms && !g.w_scale &&
         !g.A2 && !g.in_scale && g.alpha == 1.f && !(g.bias && g.residual) &&
         (!g.residual || (g.res_alpha == 1.f && g.residual == g.C && g.ldr == g.ldc)) &&
         g.lda >= g.K && g.ldw >= g.K && g.ldc >= g.N;
}

std::string gemm_key(const shai::GemmArgs& g) {
  char buf[256];
  snprintf(buf, sizeof(buf), "%d:%d,%d,%d,b%d,g%d|%d,%d,%d,%d,%d,%d,%d,%d,%d", g.conv, g.M, g.N, g.K, g.batch, g.glu,
           g.Nimg, g.H, g.Wd, g.Cin, g.Cin1, g.KH, g.stride, g.upsample, g.A2 != nullptr);
  // library-eligible problems (plain GEMM, bias at most) race hipBLASLt in the tuner, so their winner must
  // not be reused by a same-shape problem with a fused epilogue (and vice versa): separate key class
  // a folded-LayerNorm GEMM (row_mr) runs only unsplit on v4: it tunes and caches apart from the plain problem
  return std::string(buf) + (g.rms ? "|rms" : "") + (g.w_scale ? "|fp8w" : "") + (g.row_mr ? "|ln" : "") +
         (g.w_slice_rows ? "|wslice" + std::to_string(g.w_slice_rows) : "") +
         (lib_supported(g) && !g.residual ? "|lib" : "");
}

// Prefill GEMMs see a different row count every step (packed varlen prefill: M = tokens in the step), so a
// tuned choice is also filed under the row-count bucket (64 < M: 96, 128, 192, 256, 384, ...) and reused for
// every later M of that bucket instead of re-tuning per M.  Convolutions (M from the image geometry) and
// decode-sized problems (M <= 64) keep exact keys.
int m_bucket(int M) {
  if (M <= 64) return M;
  long p = 64;
  while (p < M) {
    if (p + p / 2 >= M) return (int)(p + p / 2);
    p *= 2;
  }
  return (int)p;
}

std::string gemm_bucket_key(const shai::GemmArgs& g) {
  if (g.conv || g.M <= 64) return std::string();
  shai::GemmArgs b = g;
  b.M = m_bucket(g.M);
  return gemm_key(b) + "|mbucket";
}

// exact key first, then the M bucket (a bucket hit is filed under the exact key too).  Caller holds no lock.
bool lib_enabled();
constexpr int kLibCfgId = 2000;  // = kLibCfg (below)

bool lookup_choice(const shai::GemmArgs& g, const std::string& key, Choice* out) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  // a cached library choice counts as untuned while the library path is off (the tuner races it afresh)
  auto usable = [](const Choice& c) { return c.cfg != kLibCfgId || lib_enabled(); };
  auto it = g_tuned.find(key);
  if (it != g_tuned.end() && usable(it->second)) {
    *out = it->second;
    return true;
  }
  const std::string bk = gemm_bucket_key(g);
  if (bk.empty()) return false;
  it = g_tuned.find(bk);
  if (it == g_tuned.end() || !usable(it->second)) return false;
  *out = it->second;
  g_tuned[key] = it->second;
  return true;
}

void store_choice(const shai::GemmArgs& g, const std::string& key, const Choice& c) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  g_tuned[key] = c;
  const std::string bk = gemm_bucket_key(g);
  if (!bk.empty() && !g_tuned.count(bk)) g_tuned[bk] = c;
}

bool skinny2_enabled() {  // SHAI_SKINNY2=0 keeps the wide skinny kernel out of the tuner (A/B)
  static const bool on = [] {
    const char* e = getenv("SHAI_SKINNY2");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool autotune_enabled() {
  static const bool on = [] {
    const char* e = getenv("SHAI_GEMM_AUTOTUNE");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool lib_enabled() {  // off by default: every GEMM runs on the hand-written kernels; SHAI_GEMM_LIB=1 lets the
                      // tuner race hipBLASLt again (A/B) and honours cached library choices
  static const bool on = [] {
    const char* e = getenv("SHAI_GEMM_LIB");
    return e && e[0] == '1';
  }();
  return on;
}

int max_splits_for(const shai::GemmArgs& g) {
  const int batch = g.batch > 0 ? g.batch : 1;
  if (batch != 1 || g.row_mr != nullptr) return 1;  // folded LayerNorm: applied by the unsplit v4 epilogue only
  const long kt = (g.K + 63) / 64;
  int s = 1;
  while (s < 16 && kt / (s * 2) >= 4) s *= 2;
  return s;
}

// Choice.cfg of the skinny streaming kernel (csrc/kernels/gemv.hip); Choice.splits = its K-group count
constexpr int kSkinnyCfg = 1000;
// same kernel, split-K partials reduced inside the launch by the last-arriving K group of each tile
// (no separate fold kernel); tuned against the fold form per shape
constexpr int kSkinnyFixCfg = 1100;
// Choice.cfg of the wide skinny kernel (csrc/kernels/gemv2.hip, 128-row W tiles); Choice.splits = K groups
constexpr int kSkinny2Cfg = 1200;
// the same kernel with a 6-stage ring (one workgroup per CU, deeper prefetch)
constexpr int kSkinny2DeepCfg = 1250;
inline bool is_skinny2(int cfg) { return cfg == kSkinny2Cfg || cfg == kSkinny2DeepCfg; }
inline bool is_skinny(int cfg) { return cfg == kSkinnyCfg || cfg == kSkinnyFixCfg || is_skinny2(cfg); }

// Last resort when neither the tuner nor the planner produced a usable config: an explicit, directly tested
// config, never "whichever kernel happens to be numbered highest".  The v2 128x64 tile (cfg 4) runs every
// problem the v2 kernel accepts; folded-LayerNorm problems (row_mr) are applied only by the v4 epilogue
// (cfg 9 / 10, 256 x 256 / 256 x 320).  tests/test_gemm3_gpu.py forces each of these.
Choice fallback_choice(const shai::GemmArgs& g) {
  for (int c : {4, 9, 10})
    if (shai::gemm2_cfg_supported(g, c)) return Choice{c, 1};
  return Choice{4, 1};
}

bool stream_capturing() {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  hipStreamIsCapturing(stream(), &cs);
  return cs != hipStreamCaptureStatusNone;
}

void launch_skinny2_choice(const shai::GemmArgs& g, const Tensor& like, int kg, bool deep) {
  Tensor ws;
  float* wsp = nullptr;
  const size_t bytes = shai::skinny2_workspace_bytes(g, kg);
  if (bytes > 0) {
    ws = at::empty({(long)(bytes / sizeof(float))}, like.options().dtype(at::kFloat));
    wsp = ws.data_ptr<float>();
  }
  shai::launch_skinny2(g, wsp, kg, deep, stream());
}

void launch_skinny_choice(const shai::GemmArgs& g, const Tensor& like, int kg, bool fixup) {
  Tensor ws;
  float* wsp = nullptr;
  const size_t bytes = shai::skinny_workspace_bytes_kg(g, kg);
  if (bytes > 0) {
    ws = at::empty({(long)(bytes / sizeof(float))}, like.options().dtype(at::kFloat));
    wsp = ws.data_ptr<float>();
  }
  shai::launch_skinny_kg(g, wsp, kg, stream(), fixup);
}

// Choice.cfg of the library path: plain GEMMs (no fused epilogue beyond a bias or an unscaled residual) may
// go to hipBLASLt through at::mm_out / at::addmm_out when the autotuner measures it faster than the tile
// configs -- the hand-written kernels keep every fused-epilogue / conv / GLU / gated problem.
constexpr int kLibCfg = kLibCfgId;


void launch_lib(const shai::GemmArgs& g, const Tensor& like) {
  const auto opt = like.options().dtype(at::kBFloat16);
  Tensor A = at::from_blob(const_cast<shai::bf16_t*>(g.A), {(long)g.M, (long)g.K}, {g.lda, 1L}, opt);
  Tensor W = at::from_blob(const_cast<shai::bf16_t*>(g.W), {(long)g.N, (long)g.K}, {g.ldw, 1L}, opt);
  Tensor C = at::from_blob(g.C, {(long)g.M, (long)g.N}, {g.ldc, 1L}, opt);
  if (g.residual) {          // in place: C = C + A W^T (the residual IS the output buffer)
    C.addmm_(A, W.t());
  } else if (g.bias) {
    Tensor b = at::from_blob(const_cast<shai::bf16_t*>(g.bias), {(long)g.N}, opt);
    at::addmm_out(C, b, A, W.t());
  } else {
    at::mm_out(C, A, W.t());
  }
}

void launch_choice(const shai::GemmArgs& g, const Tensor& like, Choice c) {
  if (c.cfg == kLibCfg) {
    if (lib_supported(g)) {
      launch_lib(g, like);
      return;
    }
    // the cache key does not encode the epilogue: a problem of the same shape with a fused epilogue
    // falls back to the planner's tile config
    shai::gemm2_plan(g, &c.cfg, &c.splits);
    if (!shai::gemm2_cfg_supported(g, c.cfg)) c = fallback_choice(g);
  }
  if (is_skinny2(c.cfg) && shai::skinny2_supported(g)) {
    launch_skinny2_choice(g, like, c.splits, c.cfg == kSkinny2DeepCfg);
    return;
  }
  if (is_skinny(c.cfg)) {
    if (shai::skinny_supported(g)) {
      launch_skinny_choice(g, like, c.splits, c.cfg == kSkinnyFixCfg);
      return;
    }
    shai::gemm2_plan(g, &c.cfg, &c.splits);
  }
  // a choice reused from another row count of the same bucket must still fit this problem
  if (!shai::gemm2_cfg_supported(g, c.cfg)) c = fallback_choice(g);
  Tensor ws;
  float* wsp = nullptr;
  if (c.splits > 1) {
    ws = at::empty({(long)c.splits * g.M * g.N}, like.options().dtype(at::kFloat));
    wsp = ws.data_ptr<float>();
  }
  shai::launch_gemm2_cfg(g, wsp, c.cfg, c.splits, stream());
}

// Evicts the Infinity Cache / L2 contents before a cold-cache timing: reads a 512 MB zeroed scratch buffer
// (clean lines, so the timed kernel does not pay for write-backs of the flush).
void flush_device_caches(hipStream_t st) {
  static void* buf = nullptr;
  constexpr size_t kBytes = size_t(512) << 20;
  if (buf == nullptr) {
    if (hipMalloc(&buf, kBytes + 256) != hipSuccess) {
      buf = nullptr;
      return;
    }
    (void)hipMemsetAsync(buf, 0, kBytes + 256, st);
    shai::launch_cache_flush(buf, kBytes, reinterpret_cast<unsigned*>(static_cast<char*>(buf) + kBytes), st);
  }
  shai::launch_cache_flush(buf, kBytes, reinterpret_cast<unsigned*>(static_cast<char*>(buf) + kBytes), st);
}

// Candidates are timed into a scratch output so that in-place epilogues (C aliasing
// the residual, e.g. x = x + gate * f(x)) are applied exactly once, by the caller's
// final launch.  skinny_only: the problem has an epilogue only the skinny kernel implements
// (folded RMSNorm), so only its K-group counts are candidates.
Choice tune(const shai::GemmArgs& g_real, const Tensor& like, bool skinny_only = false) {
  shai::GemmArgs g = g_real;
  const long n_out = g.glu ? g.N / 2 : g.N;
  const int nb = g.batch > 0 ? g.batch : 1;
  Tensor scratch = at::empty({(long)nb * g.M * n_out + 8}, like.options().dtype(at::kBFloat16));
  g.C = reinterpret_cast<shai::bf16_t*>(scratch.data_ptr());
  g.ldc = n_out;
  g.batch_c = (long)g.M * n_out;
  Choice def{kSkinnyCfg, shai::skinny_kgroups(g)};
  std::vector<Choice> cands;
  if (!skinny_only) {
    shai::gemm2_plan(g, &def.cfg, &def.splits);
    const int ms = max_splits_for(g);
    for (int c = 0; c < shai::gemm2_num_cfgs(); ++c) {
      if (!shai::gemm2_cfg_candidate(c) || !shai::gemm2_cfg_supported(g, c)) continue;
      for (int s = 1; s <= (shai::gemm2_cfg_splittable(c) ? ms : 1); s *= 2) cands.push_back({c, s});
    }
  }
  if (shai::skinny_supported(g))
    for (int kg = 1; kg <= shai::skinny_max_kgroups(g); kg *= 2) {
      cands.push_back({kSkinnyCfg, kg});
      if (kg > 1) cands.push_back({kSkinnyFixCfg, kg});
    }
  if (shai::skinny2_supported(g) && skinny2_enabled())
    for (int kg = 1; kg <= shai::skinny2_max_kgroups(g); kg *= 2) {
      cands.push_back({kSkinny2Cfg, kg});
      cands.push_back({kSkinny2DeepCfg, kg});
    }
  // residual epilogues are in place (C aliases the residual): timing them into the scratch output is not
  // equivalent, so only bias-or-nothing problems race the library
  if (!skinny_only && lib_enabled() && lib_supported(g_real) && !g_real.residual) cands.push_back({kLibCfg, 1});
  hipStream_t st = stream();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  Choice best = def;
  float best_ms = 1e30f;
  // Decode-shaped problems (M <= 64) stream weights that are NOT cache resident in a real decode step (the
  // model's weights are tens of GB; the MALL holds 256 MB): each timed launch runs behind a flush of the
  // Infinity Cache so the candidates are ranked by their HBM-streaming speed, not by a warm-cache replay.
  const bool cold = g.M <= 64 && (long)g.N * g.K * (g.w_scale ? 1 : 2) >= (4L << 20);
  for (const Choice& c : cands) {
    launch_choice(g, like, c);  // warm (also instantiates caches)
    float ms = 0.f;
    if (cold) {  // median of 5 single cold launches
      float ts[5];
      for (int r = 0; r < 5; ++r) {
        flush_device_caches(st);
        hipEventRecord(e0, st);
        launch_choice(g, like, c);
        hipEventRecord(e1, st);
        hipEventSynchronize(e1);
        ts[r] = 0.f;
        hipEventElapsedTime(&ts[r], e0, e1);
      }
      std::sort(ts, ts + 5);
      ms = ts[2];
    } else {
      hipEventRecord(e0, st);
      for (int r = 0; r < 3; ++r) launch_choice(g, like, c);
      hipEventRecord(e1, st);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
    }
    if (ms < best_ms) {
      best_ms = ms;
      best = c;
    }
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return best;
}

// Skinny-kernel-only problems (folded RMSNorm epilogue): tuned over the K-group count.
void run_skinny(const shai::GemmArgs& g, const Tensor& like) {
  const std::string key = gemm_key(g);
  Choice c{-1, 1};
  if (!lookup_choice(g, key, &c) || !is_skinny(c.cfg)) c = Choice{-1, 1};
  if (c.cfg < 0) {
    if (!stream_capturing() && autotune_enabled()) {
      c = tune(g, like, true);
      store_choice(g, key, c);
    } else {
      c = Choice{kSkinnyCfg, shai::skinny_kgroups(g)};
    }
  }
  launch_choice(g, like, c);
}

// Statistics of the GEMM output wanted by the next norm: GroupNorm col partials [M / 128, N, 2] and / or LayerNorm
// row moments [M, 2] = (mean, rstd).  The v4 wide epilogue writes them when the final choice runs it on every tile
// (gemm4_stats_ok); otherwise a pass over the output produces the same statistics.
struct OutStats {
  float* gn_part = nullptr;
  float* ln_mr = nullptr;
  float ln_eps = 1e-5f;
  bool any() const { return gn_part != nullptr || ln_mr != nullptr; }
};

void launch_final(shai::GemmArgs g, const Tensor& like, const Choice& c, const OutStats* st) {
  if (st == nullptr || !st->any()) {
    launch_choice(g, like, c);
    return;
  }
  int bm = 0, bn = 0;
  bool v4 = c.cfg >= 0 && c.cfg < shai::gemm2_num_cfgs() && c.splits <= 1 && shai::gemm2_cfg_supported(g, c.cfg);
  if (v4) {
    shai::gemm2_cfg_info(c.cfg, &bm, &bn);
    v4 = (bm == 8 || bm == 9) && bn < 0 && shai::gemm4_stats_ok(g, -bn);
  }
  Tensor rp;
  if (v4) {
    g.col_part = st->gn_part;
    if (st->ln_mr) {
      g.row_part_slots = 4 * (g.N / -bn);
      rp = at::empty({(long)g.M * g.row_part_slots * 2}, like.options().dtype(at::kFloat));
      g.row_part = rp.data_ptr<float>();
    }
  }
  launch_choice(g, like, c);
  if (st->gn_part && g.col_part == nullptr) shai::launch_col_partials(g.C, g.M, g.N, g.ldc, st->gn_part, stream());
  if (st->ln_mr) {
    if (g.row_part) shai::launch_row_moments_from_partials(g.row_part, g.M, g.row_part_slots, g.N, st->ln_eps,
                                                           st->ln_mr, stream());
    else shai::launch_row_moments(g.C, g.M, g.N, g.ldc, st->ln_eps, st->ln_mr, stream());
  }
}

void run_gemm(const shai::GemmArgs& g, const Tensor& like, long a_bytes, long w_bytes, long a2_bytes,
              const OutStats* st = nullptr) {
  static const int forced = [] {  // tests / tools: pin one config for every supported GEMM/conv
    const char* e = getenv("SHAI_GEMM_FORCE");
    return e ? atoi(e) : -1;
  }();
  if (!use_v2(g, a_bytes, w_bytes, a2_bytes)) {
    SHAI_CHECK(g.gate == nullptr, "gated GEMM epilogue needs the v2 kernel (operands < 2 GiB, SHAI_GEMM_V1 unset)");
    SHAI_CHECK(g.row_mr == nullptr, "folded LayerNorm needs the v4 kernel (operands < 2 GiB, SHAI_GEMM_V1 unset)");
    SHAI_CHECK(g.w_slice_rows == 0, "weight slices need the v4 kernel (operands < 2 GiB, SHAI_GEMM_V1 unset)");
    if (g.conv) {  // the v1 conv instantiations: activation none / silu, silu only with 64-channel sources
      const bool fast = g.Cin % 64 == 0 && (g.A2 == nullptr || g.Cin1 % 64 == 0);
      SHAI_CHECK(!g.glu && (g.act == 0 || (g.act == 1 && fast)), "conv2d output activation ", g.act,
                 " is not implemented for this input layout");
    }
    shai::launch_gemm(g, stream());
    if (st && st->any()) {  // v1 writes no statistics
      if (st->gn_part) shai::launch_col_partials(g.C, g.M, g.N, g.ldc, st->gn_part, stream());
      if (st->ln_mr) shai::launch_row_moments(g.C, g.M, g.N, g.ldc, st->ln_eps, st->ln_mr, stream());
    }
    return;
  }
  static const int forced_splits = [] {  // with SHAI_GEMM_FORCE: split-K count (clamped to the problem's maximum)
    const char* e = getenv("SHAI_GEMM_FORCE_SPLITS");
    return e ? std::max(1, atoi(e)) : 1;
  }();
  if (forced >= 0 && forced < shai::gemm2_num_cfgs() && shai::gemm2_cfg_supported(g, forced)) {
    const int sp = shai::gemm2_cfg_splittable(forced) ? std::min(forced_splits, max_splits_for(g)) : 1;
    launch_final(g, like, Choice{forced, sp}, st);
    return;
  }
  const std::string key = gemm_key(g);
  Choice c{-1, 1};
  if (!lookup_choice(g, key, &c)) c = Choice{-1, 1};
  if (c.cfg < 0) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hipStreamIsCapturing(stream(), &cs);
    if (cs == hipStreamCaptureStatusNone && autotune_enabled()) {
      c = tune(g, like);
      store_choice(g, key, c);
    } else {
      if (shai::skinny_supported(g)) {
        c = Choice{kSkinnyCfg, shai::skinny_kgroups(g)};
      } else {
        shai::gemm2_plan(g, &c.cfg, &c.splits);
        if (!shai::gemm2_cfg_supported(g, c.cfg)) c = fallback_choice(g);
      }
    }
  }
  if (g.row_mr != nullptr) c.splits = 1;  // a cached choice of the plain problem with this key may be split
  launch_final(g, like, c, st);
}

std::vector<std::string> gemm_tuning_table() {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  std::vector<std::string> out;
  for (auto& kv : g_tuned) {
    if (is_skinny(kv.second.cfg)) {
      out.push_back(kv.first + " -> skinny kg=" + std::to_string(kv.second.splits) +
                    (kv.second.cfg == kSkinnyFixCfg ? " (in-kernel fixup)" : ""));
      continue;
    }
    if (kv.second.cfg == kLibCfg) {
      out.push_back(kv.first + " -> hipblaslt");
      continue;
    }
    int bm, bn;
    shai::gemm2_cfg_info(kv.second.cfg, &bm, &bn);
    out.push_back(kv.first + " -> " + std::to_string(bm) + "x" + std::to_string(bn) + " splitk=" +
                  std::to_string(kv.second.splits));
  }
  return out;
}

const shai::bf16_t* cptr(const Tensor& t) { return reinterpret_cast<const shai::bf16_t*>(t.data_ptr()); }
shai::bf16_t* mptr(const Tensor& t) { return reinterpret_cast<shai::bf16_t*>(t.data_ptr()); }
const shai::bf16_t* optr(const optional<Tensor>& t) { return t.has_value() ? cptr(*t) : nullptr; }

void check_bf16(const Tensor& t, const char* name) {
  SHAI_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  SHAI_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16, got ", t.scalar_type());
  SHAI_CHECK(t.stride(-1) == 1, name, " last dim must be contiguous");
  SHAI_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}
void check_f32(const Tensor& t, const char* name) {
  SHAI_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), name, " must be contiguous f32 GPU");
}
void check_i32(const Tensor& t, const char* name) {
  SHAI_CHECK(t.is_cuda() && t.scalar_type() == at::kInt && t.is_contiguous(), name, " must be contiguous int32 GPU");
}
void check_rows(const Tensor& t, const char* name) {
  check_bf16(t, name);
  for (int d = 0; d + 1 < t.dim(); ++d) SHAI_CHECK(t.stride(d) % 8 == 0 || t.size(d) == 1, name, " stride not 16B aligned");
}

// ---------------------------------------------------------------- norms
void rmsnorm(const Tensor& x, const optional<Tensor>& w, const Tensor& out, const optional<Tensor>& residual,
             const optional<Tensor>& residual_out, double eps, double w_offset) {
  check_rows(x, "x");
  check_rows(out, "out");
  const int D = x.size(-1);
  SHAI_CHECK(D % 8 == 0 && D <= 8192, "rmsnorm D must be a multiple of 8 and <= 8192");
  const long rows = x.numel() / D;
  SHAI_CHECK(x.dim() == 2 || x.is_contiguous(), "rmsnorm x must be 2D strided or contiguous");
  shai::RowNormArgs a{};
  a.x = cptr(x);
  a.w = optr(w);
  a.out = mptr(out);
  if (residual) {
    SHAI_CHECK(residual->is_contiguous() && x.is_contiguous(), "residual path needs contiguous tensors");
    a.residual = cptr(*residual);
    a.residual_out = residual_out ? mptr(*residual_out) : nullptr;
  }
  a.rows = rows;
  a.D = D;
  a.x_stride = x.dim() == 2 ? x.stride(0) : D;
  a.out_stride = out.dim() == 2 ? out.stride(0) : D;
  a.eps = eps;
  a.w_offset = w_offset;
  shai::launch_rmsnorm(a, stream());
}

void layernorm(const Tensor& x, const optional<Tensor>& w, const optional<Tensor>& b, const Tensor& out,
               const optional<Tensor>& residual, const optional<Tensor>& residual_out, double eps) {
  check_rows(x, "x");
  check_rows(out, "out");
  const int D = x.size(-1);
  SHAI_CHECK(D % 8 == 0 && D <= 8192, "layernorm D must be a multiple of 8 and <= 8192");
  SHAI_CHECK(x.dim() == 2 || x.is_contiguous(), "layernorm x must be 2D strided or contiguous");
  shai::RowNormArgs a{};
  a.x = cptr(x);
  a.w = optr(w);
  a.b = optr(b);
  a.out = mptr(out);
  if (residual) {
    SHAI_CHECK(residual->is_contiguous() && x.is_contiguous(), "residual path needs contiguous tensors");
    a.residual = cptr(*residual);
    a.residual_out = residual_out ? mptr(*residual_out) : nullptr;
  }
  a.rows = x.numel() / D;
  a.D = D;
  a.x_stride = x.dim() == 2 ? x.stride(0) : D;
  a.out_stride = out.dim() == 2 ? out.stride(0) : D;
  a.eps = eps;
  a.w_offset = 0.f;
  shai::launch_layernorm(a, stream());
}

// y = LayerNorm(x) * (1 + scale[r / rows_per_mod]) + shift[r / rows_per_mod]  (AdaLN modulation, no affine)
void layernorm_mod(const Tensor& x, const Tensor& scale, const Tensor& shift, const Tensor& out,
                   int64_t rows_per_mod, double eps) {
  check_rows(x, "x");
  check_rows(out, "out");
  check_bf16(scale, "scale");
  check_bf16(shift, "shift");
  const int D = x.size(-1);
  SHAI_CHECK(D % 8 == 0 && D <= 8192, "layernorm_mod D must be a multiple of 8 and <= 8192");
  SHAI_CHECK(x.dim() == 2 || x.is_contiguous(), "layernorm_mod x must be 2D strided or contiguous");
  SHAI_CHECK(scale.dim() == 2 && shift.dim() == 2 && scale.size(1) == D && shift.size(1) == D &&
                 scale.stride(0) == shift.stride(0) && scale.stride(0) % 8 == 0,
             "scale/shift must be [G, D] with equal 16B-aligned row strides");
  const long rows = x.numel() / D;
  SHAI_CHECK(rows_per_mod > 0 && scale.size(0) * rows_per_mod >= rows, "modulation rows");
  shai::RowNormArgs a{};
  a.x = cptr(x);
  a.w = cptr(scale);
  a.b = cptr(shift);
  a.out = mptr(out);
  a.rows = rows;
  a.D = D;
  a.x_stride = x.dim() == 2 ? x.stride(0) : D;
  a.out_stride = out.dim() == 2 ? out.stride(0) : D;
  a.eps = eps;
  a.w_offset = 1.f;
  a.rows_per_w = rows_per_mod;
  a.w_stride = scale.stride(0);
  shai::launch_layernorm(a, stream());
}

// In-place per-head RMSNorm(q), RMSNorm(k) + pair RoPE on a packed QKV buffer [rows, >= 2*H*D].
void qk_norm_rope(const Tensor& x, const optional<Tensor>& q_w, const optional<Tensor>& k_w,
                  const optional<Tensor>& cos, const optional<Tensor>& sin, int64_t H, int64_t D, int64_t S,
                  double eps) {
  check_bf16(x, "x");
  SHAI_CHECK(x.dim() == 2 && x.size(1) >= 2 * H * D && x.stride(0) % 2 == 0, "qk_norm_rope x [rows, >= 2*H*D]");
  SHAI_CHECK(D % 2 == 0 && D <= 128, "qk_norm_rope head dim must be even and <= 128");
  SHAI_CHECK(cos.has_value() == sin.has_value(), "cos and sin go together");
  if (q_w) { check_bf16(*q_w, "q_w"); SHAI_CHECK(q_w->numel() == D, "q_w [D]"); }
  if (k_w) { check_bf16(*k_w, "k_w"); SHAI_CHECK(k_w->numel() == D, "k_w [D]"); }
  if (cos) {
    check_f32(*cos, "cos");
    check_f32(*sin, "sin");
    SHAI_CHECK(cos->numel() == S * D / 2 && sin->numel() == S * D / 2, "cos/sin must be [S, D/2]");
  }
  SHAI_CHECK(S > 0, "S > 0");
  shai::launch_qk_norm_rope(mptr(x), x.stride(0), x.size(0), S, H, D, optr(q_w), optr(k_w),
                            cos ? cos->data_ptr<float>() : nullptr, sin ? sin->data_ptr<float>() : nullptr, eps,
                            stream());
}

// x [N, HW, C1] (+ x2 [N, HW, C - C1]: channels of a virtual concat); counters: optional zeroed int32 [>= N]
// tickets -> finalize fused into the stats launch.
static void gn_sources(const Tensor& x, const optional<Tensor>& x2, shai::GroupNormArgs& a, int* C) {
  check_bf16(x, "x");
  SHAI_CHECK(x.is_contiguous() && x.dim() == 3, "groupnorm x must be contiguous [N, HW, C]");
  *C = x.size(2);
  a.C1 = x.size(2);
  if (x2.has_value()) {
    check_bf16(*x2, "x2");
    SHAI_CHECK(x2->is_contiguous() && x2->dim() == 3 && x2->size(0) == x.size(0) && x2->size(1) == x.size(1),
               "groupnorm x2 must be contiguous [N, HW, C2] matching x");
    SHAI_CHECK(x.size(2) % 8 == 0 && x2->size(2) % 8 == 0, "groupnorm concat halves need C % 8 == 0");
    a.x2 = cptr(*x2);
    *C += x2->size(2);
  }
}

void groupnorm_stats(const Tensor& x, const optional<Tensor>& x2, const optional<Tensor>& gamma,
                     const optional<Tensor>& beta, const Tensor& partials, const Tensor& scale, const Tensor& shift,
                     const optional<Tensor>& counters, int64_t G, double eps) {
  check_f32(partials, "partials");
  check_f32(scale, "scale");
  check_f32(shift, "shift");
  shai::GroupNormArgs a{};
  int C;
  gn_sources(x, x2, a, &C);
  const int N = x.size(0), HW = x.size(1);
  if (counters.has_value()) {
    SHAI_CHECK(counters->is_cuda() && counters->scalar_type() == at::kInt && counters->numel() >= N,
               "groupnorm counters must be int32 [>= N] on the device");
    a.counters = reinterpret_cast<unsigned*>(counters->data_ptr<int>());
  }
  SHAI_CHECK(C % 8 == 0 && C % G == 0 && C <= 4096 && G <= 128, "groupnorm: bad C/G");
  SHAI_CHECK(partials.numel() >= (long)N * shai::gn_num_blocks(N, HW, C) * G * 2, "partials too small");
  SHAI_CHECK(scale.numel() >= (long)N * C && shift.numel() >= (long)N * C, "scale/shift too small");
  a.x = cptr(x);
  a.gamma = optr(gamma);
  a.beta = optr(beta);
  a.partials = partials.data_ptr<float>();
  a.scale = scale.data_ptr<float>();
  a.shift = shift.data_ptr<float>();
  a.N = N;
  a.HW = HW;
  a.C = C;
  a.G = G;
  a.eps = eps;
  shai::launch_groupnorm_stats(a, stream());
}

// GroupNorm (scale, shift) from the col partials a GEMM / conv epilogue wrote ([Nimg * HW / 128, C, 2] per source)
void groupnorm_from_partials(const Tensor& part1, const optional<Tensor>& part2, int64_t C1, int64_t C2,
                             int64_t Nimg, int64_t HW, const optional<Tensor>& gamma, const optional<Tensor>& beta,
                             const Tensor& scale, const Tensor& shift, int64_t G, double eps) {
  check_f32(part1, "part1");
  check_f32(scale, "scale");
  check_f32(shift, "shift");
  const long C = C1 + C2;
  SHAI_CHECK(HW % 128 == 0 && C % G == 0 && G <= 128 && C <= 8192, "groupnorm_from_partials: bad HW / C / G");
  SHAI_CHECK(part1.numel() == Nimg * HW / 128 * C1 * 2, "part1 must be [Nimg * HW / 128, C1, 2]");
  if (part2.has_value()) {
    check_f32(*part2, "part2");
    SHAI_CHECK(part2->numel() == Nimg * HW / 128 * C2 * 2, "part2 must be [Nimg * HW / 128, C2, 2]");
  } else {
    SHAI_CHECK(C2 == 0, "C2 > 0 needs part2");
  }
  SHAI_CHECK(scale.numel() >= Nimg * C && shift.numel() >= Nimg * C, "scale/shift too small");
  shai::launch_gn_from_partials(part1.data_ptr<float>(), C1, part2 ? part2->data_ptr<float>() : nullptr, C2, Nimg,
                                HW, G, optr(gamma), optr(beta), eps, scale.data_ptr<float>(), shift.data_ptr<float>(),
                                stream());
}

// the statistics passes on their own (tests, and producers outside the GEMM kernels)
void col_partials(const Tensor& x, const Tensor& part) {
  check_rows(x, "x");
  check_f32(part, "part");
  SHAI_CHECK(x.dim() == 2, "col_partials: x must be 2D [M, N]");
  const long M = x.size(0);
  const int N = x.size(1);
  SHAI_CHECK(M % 128 == 0 && N % 8 == 0 && N <= 2048 && part.numel() == M / 128 * N * 2,
             "col_partials: M % 128 == 0, N % 8 == 0, N <= 2048, part [M / 128, N, 2]");
  shai::launch_col_partials(cptr(x), M, N, x.stride(0), part.data_ptr<float>(), stream());
}

void row_moments(const Tensor& x, const Tensor& mr, double eps) {
  check_rows(x, "x");
  check_f32(mr, "mr");
  SHAI_CHECK(x.dim() == 2 && x.size(1) % 8 == 0 && mr.numel() == 2 * x.size(0), "row_moments: x [M, N % 8], mr [M, 2]");
  shai::launch_row_moments(cptr(x), x.size(0), x.size(1), x.stride(0), eps, mr.data_ptr<float>(), stream());
}

void groupnorm_apply(const Tensor& x, const optional<Tensor>& x2, const Tensor& scale, const Tensor& shift,
                     const Tensor& out, bool silu) {
  check_bf16(out, "out");
  check_f32(scale, "scale");
  check_f32(shift, "shift");
  shai::GroupNormArgs a{};
  int C;
  gn_sources(x, x2, a, &C);
  SHAI_CHECK(out.is_contiguous() && out.numel() == x.size(0) * x.size(1) * (long)C, "groupnorm_apply out must be [N,HW,C]");
  SHAI_CHECK(scale.numel() >= x.size(0) * (long)C && shift.numel() >= x.size(0) * (long)C, "scale/shift too small");
  a.x = cptr(x);
  a.scale = scale.data_ptr<float>();
  a.shift = shift.data_ptr<float>();
  a.out = mptr(out);
  a.N = x.size(0);
  a.HW = x.size(1);
  a.C = C;
  SHAI_CHECK(a.C % 8 == 0, "C % 8");
  a.silu = silu;
  shai::launch_groupnorm_apply(a, stream());
}

// ---------------------------------------------------------------- GEMM
// Norm hand-off tensors of a GEMM / conv: ln_mr [M, 2] + ln_s [N] (LayerNorm of A folded in), gn_part
// [M / 128, N, 2] (GroupNorm partials of the output), ln_stats [M, 2] (LayerNorm moments of the output).
void attach_norm_io(shai::GemmArgs& g, const optional<Tensor>& ln_mr, const optional<Tensor>& ln_s,
                    const optional<Tensor>& gn_part, const optional<Tensor>& ln_stats, double ln_eps, OutStats* st) {
  if (ln_mr.has_value()) {
    SHAI_CHECK(ln_s.has_value(), "ln_mr needs ln_s");
    check_f32(*ln_mr, "ln_mr");
    check_f32(*ln_s, "ln_s");
    SHAI_CHECK(ln_mr->numel() == 2L * g.M && ln_s->numel() == g.N, "ln_mr must be [M, 2] and ln_s [N]");
    SHAI_CHECK(reinterpret_cast<uintptr_t>(ln_s->data_ptr()) % 16 == 0, "ln_s must be 16-byte aligned");
    g.row_mr = ln_mr->data_ptr<float>();
    g.col_s = ln_s->data_ptr<float>();
  }
  const int n_out = g.glu ? g.N / 2 : g.N;
  if (gn_part.has_value()) {
    check_f32(*gn_part, "gn_part");
    SHAI_CHECK(g.M % 128 == 0 && n_out % 8 == 0 && n_out <= 2048 && gn_part->numel() == (long)g.M / 128 * n_out * 2,
               "gn_part must be [M / 128, N, 2] with M % 128 == 0, N % 8 == 0, N <= 2048");
    SHAI_CHECK(reinterpret_cast<uintptr_t>(gn_part->data_ptr()) % 16 == 0, "gn_part must be 16-byte aligned");
    st->gn_part = gn_part->data_ptr<float>();
  }
  if (ln_stats.has_value()) {
    check_f32(*ln_stats, "ln_stats");
    SHAI_CHECK(ln_stats->numel() == 2L * g.M && n_out % 8 == 0, "ln_stats must be [M, 2] (N % 8 == 0)");
    st->ln_mr = ln_stats->data_ptr<float>();
    st->ln_eps = (float)ln_eps;
  }
}

// a: [M, K] or [B, M, K]; w: [N, K] or [B, N, K]; c: [M, N'] or [B, M, N'] (N' = N or N/2 for glu)
void gemm(const Tensor& a, const Tensor& w, const Tensor& c, const optional<Tensor>& bias,
          const optional<Tensor>& bias2d, int64_t rows_per_bias2d, const optional<Tensor>& residual, double alpha,
          double res_alpha, int64_t act, bool glu, const optional<Tensor>& gate, int64_t rows_per_gate,
          int64_t force_cfg, double rms_eps, const optional<Tensor>& w_scale, const optional<Tensor>& ln_mr,
          const optional<Tensor>& ln_s, const optional<Tensor>& gn_part, const optional<Tensor>& ln_stats,
          double ln_eps, int64_t w_slice_rows) {
  check_rows(a, "a");
  if (w_scale.has_value()) {  // fp8 (e4m3) weights + fp32 per-row scale: skinny (decode-shaped) kernel only
    SHAI_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat8_e4m3fn && w.dim() == 2 && w.stride(1) == 1 &&
                   w.stride(0) % 16 == 0,
               "fp8 gemm: w must be a row-major float8_e4m3fn [N, K] matrix with 16-byte aligned rows");
    check_f32(*w_scale, "w_scale");
    SHAI_CHECK(w_scale->is_contiguous() && w_scale->numel() == w.size(0), "w_scale must be fp32 [N]");
    SHAI_CHECK(a.dim() == 2 && a.size(0) <= 64 && a.size(1) % 16 == 0,
               "fp8 gemm: decode-shaped activations only (M <= 64, K % 16 == 0); dequantize for larger M");
  } else {
    check_rows(w, "w");
  }
  check_bf16(c, "c");
  SHAI_CHECK(a.dim() == w.dim() || w.dim() == 2, "gemm rank mismatch");
  const bool batched = a.dim() == 3;
  shai::GemmArgs g{};
  g.A = cptr(a);
  g.W = cptr(w);
  g.C = mptr(c);
  g.M = a.size(-2);
  g.K = a.size(-1);
  g.N = w.size(-2);
  if (w_slice_rows > 0) {  // w: [M / w_slice_rows * N, K], slice s for rows [s w_slice_rows, (s + 1) w_slice_rows)
    SHAI_CHECK(a.dim() == 2 && w.dim() == 2 && !glu && g.M % w_slice_rows == 0, "w_slice_rows: 2D, non-GLU, M % rows == 0");
    const long slices = g.M / w_slice_rows;
    SHAI_CHECK(w.size(0) % slices == 0, "w_slice_rows: w must hold M / w_slice_rows row slices");
    g.N = w.size(0) / slices;
    g.w_slice_rows = w_slice_rows;
  }
  SHAI_CHECK(w.size(-1) == g.K, "gemm K mismatch: a ", a.sizes(), " w ", w.sizes());
  SHAI_CHECK(g.K % 8 == 0, "gemm K must be a multiple of 8");
  SHAI_CHECK(c.size(-2) == g.M && c.size(-1) == (glu ? g.N / 2 : g.N), "gemm output shape mismatch ", c.sizes());
  SHAI_CHECK(!glu || g.N % 4 == 0, "glu needs N % 4 == 0");
  g.lda = a.stride(-2);
  g.ldw = w.stride(-2);
  g.ldc = c.stride(-2);
  g.batch = batched ? a.size(0) : 1;
  g.batch_a = batched ? a.stride(0) : 0;
  g.batch_w = (batched && w.dim() == 3) ? w.stride(0) : 0;
  g.batch_c = batched ? c.stride(0) : 0;
  if (bias) {
    check_bf16(*bias, "bias");
    SHAI_CHECK(bias->numel() == g.N, "bias size");
    g.bias = cptr(*bias);
  }
  if (bias2d) {
    check_bf16(*bias2d, "bias2d");
    SHAI_CHECK(bias2d->is_contiguous() && bias2d->size(-1) == g.N && rows_per_bias2d > 0, "bias2d shape");
    g.bias2d = cptr(*bias2d);
    g.rows_per_bias2d = rows_per_bias2d;
  }
  if (residual) {
    check_bf16(*residual, "residual");
    SHAI_CHECK(residual->size(-2) == g.M && residual->size(-1) == c.size(-1), "residual shape");
    g.residual = cptr(*residual);
    g.ldr = residual->stride(-2);
    g.batch_r = batched ? residual->stride(0) : 0;
  }
  if (gate) {
    check_bf16(*gate, "gate");
    SHAI_CHECK(gate->dim() == 2 && gate->size(1) == c.size(-1) && rows_per_gate > 0 &&
                   gate->size(0) * rows_per_gate >= (long)g.batch * g.M,
               "gate must be [G, N_out] with G * rows_per_gate >= rows");
    g.gate = cptr(*gate);
    g.gate_stride = gate->stride(0);
    g.rows_per_gate = rows_per_gate;
  }
  g.alpha = alpha;
  g.res_alpha = res_alpha;
  g.act = act;
  g.glu = glu;
  if (w_scale.has_value()) {
    g.w_scale = w_scale->data_ptr<float>();
    SHAI_CHECK(shai::skinny_supported(g), "fp8 gemm: problem not supported by the skinny kernel");
    if (rms_eps >= 0) {
      g.rms = 1;
      g.rms_eps = (float)rms_eps;
    }
    SHAI_CHECK(force_cfg < 0 || (force_cfg >= kSkinnyCfg && force_cfg <= kSkinnyCfg + 64) ||
                   (force_cfg > kSkinnyFixCfg && force_cfg <= kSkinnyFixCfg + 64),
               "fp8 gemm: force_cfg must be 1000 (+ kg) or 1100 + kg (1 <= kg <= 64): only the skinny kernel takes "
               "fp8 weights");
    if (force_cfg > kSkinnyFixCfg) launch_choice(g, a, Choice{kSkinnyFixCfg, (int)(force_cfg - kSkinnyFixCfg)});
    else if (force_cfg > kSkinnyCfg) launch_choice(g, a, Choice{kSkinnyCfg, (int)(force_cfg - kSkinnyCfg)});
    else run_skinny(g, a);
    return;
  }
  const long a_bytes = (batched ? (long)a.size(0) * a.stride(0) : (long)g.M * g.lda) * 2;
  // tests / tools bypass the tuner: force_cfg = gemm2 config, 1000 = skinny kernel (heuristic K groups),
  // 1000 + kg = skinny kernel with kg K groups (separate fold), 1100 + kg = the same with the in-kernel fixup
  // 1200 + kg = the wide skinny kernel (gemv2.hip) with kg K groups (in-kernel fixup), 1250 + kg its 6-stage form
  const bool force_s2d = force_cfg > kSkinny2DeepCfg && force_cfg < kLibCfg;
  const bool force_s2 = force_cfg > kSkinny2Cfg && force_cfg < kLibCfg;
  const bool force_skinny = force_cfg >= kSkinnyCfg && force_cfg != kLibCfg;
  const bool force_fix = force_cfg > kSkinnyFixCfg && force_cfg != kLibCfg && !force_s2;
  const int force_kg = force_s2d  ? (int)(force_cfg - kSkinny2DeepCfg)
                       : force_s2 ? (int)(force_cfg - kSkinny2Cfg)
                       : force_fix ? (int)(force_cfg - kSkinnyFixCfg)
                       : force_cfg > kSkinnyCfg ? (int)(force_cfg - kSkinnyCfg)
                                                : shai::skinny_kgroups(g);
  const int force_skcfg = force_s2d ? kSkinny2DeepCfg : force_s2 ? kSkinny2Cfg : force_fix ? kSkinnyFixCfg : kSkinnyCfg;
  if (rms_eps >= 0) {
    // RMSNorm(a) folded in (norm gain pre-multiplied into w): fused into the skinny kernel for
    // decode-shaped problems, otherwise an explicit unweighted RMSNorm pass feeds the GEMM.
    SHAI_CHECK(!batched, "folded RMSNorm needs a 2D activation");
    if (shai::skinny_supported(g) && (force_cfg < 0 || force_skinny)) {
      g.rms = 1;
      g.rms_eps = (float)rms_eps;
      if (force_skinny) launch_choice(g, a, Choice{force_skcfg, force_kg});
      else run_skinny(g, a);
      return;
    }
    Tensor xn = at::empty({g.M, g.K}, a.options());
    shai::RowNormArgs r{};
    r.x = cptr(a);
    r.out = mptr(xn);
    r.rows = g.M;
    r.D = g.K;
    r.x_stride = g.lda;
    r.out_stride = g.K;
    r.eps = rms_eps;
    SHAI_CHECK(g.K % 8 == 0 && g.K <= 8192, "folded RMSNorm: K must be a multiple of 8 and <= 8192");
    shai::launch_rmsnorm(r, stream());
    g.A = cptr(xn);
    g.lda = g.K;
    run_gemm(g, xn, (long)g.M * g.K * 2, (long)g.N * g.ldw * 2, 0);
    return;
  }
  if (ln_mr.has_value() || gn_part.has_value() || ln_stats.has_value()) {
    SHAI_CHECK(!batched && g.gate == nullptr &&
                   (force_cfg < 0 || force_cfg < shai::gemm2_num_cfgs() || (force_cfg >= 3000 && force_cfg < 4000)),
               "folded LayerNorm / output statistics: 2D, ungated GEMMs on the tile kernels");
    SHAI_CHECK(!glu || (!gn_part.has_value() && !ln_stats.has_value()), "output statistics of a GLU GEMM");
    OutStats st;
    attach_norm_io(g, ln_mr, ln_s, gn_part, ln_stats, ln_eps, &st);
    if (force_cfg >= 3000) {  // tests: a split-K tile choice (the fold writes the GroupNorm partials)
      const int cfg = (int)((force_cfg - 3000) % 100), splits = (int)((force_cfg - 3000) / 100);
      SHAI_CHECK(cfg < shai::gemm2_num_cfgs() && shai::gemm2_cfg_supported(g, cfg) && splits >= 1, "bad forced split");
      launch_final(g, a, Choice{cfg, splits}, &st);
    } else if (force_cfg >= 0) {
      SHAI_CHECK(shai::gemm2_cfg_supported(g, force_cfg), "bad force_cfg");
      launch_final(g, a, Choice{(int)force_cfg, 1}, &st);
    } else {
      run_gemm(g, a, a_bytes, (long)g.N * g.ldw * 2, 0, &st);
    }
    return;
  }
  if (force_cfg >= 3000 && force_cfg < 4000) {  // tests: tile config (force % 100) with (force - 3000) / 100 K splits
    const int cfg = (int)((force_cfg - 3000) % 100), splits = (int)((force_cfg - 3000) / 100);
    SHAI_CHECK(cfg < shai::gemm2_num_cfgs() && shai::gemm2_cfg_supported(g, cfg) && splits >= 1 && !batched,
               "bad forced split config");
    launch_choice(g, a, Choice{cfg, splits});
    return;
  }
  if (force_cfg == kLibCfg) {  // tests: pin the hipBLASLt path
    SHAI_CHECK(lib_supported(g), "library GEMM path does not support this problem's epilogue");
    launch_lib(g, a);
    return;
  }
  if (force_cfg >= 0) {
    if (force_skinny) {
      SHAI_CHECK((force_s2 ? shai::skinny2_supported(g) : shai::skinny_supported(g)) && force_kg >= 1 &&
                     force_kg <= 64,
                 "skinny kernel does not support this problem");
      launch_choice(g, a, Choice{force_skcfg, force_kg});
    } else {
      SHAI_CHECK(force_cfg < shai::gemm2_num_cfgs() && shai::gemm2_cfg_supported(g, force_cfg), "bad force_cfg");
      launch_choice(g, a, Choice{(int)force_cfg, 1});
    }
    return;
  }
  run_gemm(g, a, a_bytes, (long)g.N * g.ldw * 2, 0);
}

// x: [N, H, W, C1] NHWC; x2 optional [N, H, W, C2]; w: [Cout, KH*KW*Cin]; out: [N, OH, OW, Cout]
void conv2d(const Tensor& x, const optional<Tensor>& x2, const Tensor& w, const Tensor& out,
            const optional<Tensor>& bias, const optional<Tensor>& bias2d, const optional<Tensor>& residual,
            const optional<Tensor>& in_scale, const optional<Tensor>& in_shift, int64_t in_act, int64_t kh,
            int64_t kw, int64_t stride, int64_t pad, bool upsample, int64_t act, double res_alpha,
            const optional<Tensor>& ln_mr, const optional<Tensor>& ln_s, const optional<Tensor>& gn_part,
            const optional<Tensor>& ln_stats, double ln_eps, bool up_phases) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_bf16(out, "out");
  SHAI_CHECK(x.is_contiguous() && out.is_contiguous() && w.is_contiguous(), "conv2d needs contiguous tensors");
  SHAI_CHECK(x.dim() == 4 && out.dim() == 4, "conv2d needs NHWC 4D tensors");
  shai::GemmArgs g{};
  g.conv = 1;
  g.Nimg = x.size(0);
  g.H = x.size(1);
  g.Wd = x.size(2);
  g.Cin1 = x.size(3);
  g.Cin = g.Cin1;
  // concat fallback: the fused two-source gather of the tile kernels (v4 / four-wave / v2) needs both sources at
  // multiples of 64 channels, so a 64-deep K-tile never straddles the split (every SD2.1 skip concat qualifies)
  Tensor xcat;
  if (x2) {
    check_bf16(*x2, "x2");
    SHAI_CHECK(x2->is_contiguous() && x2->size(0) == g.Nimg && x2->size(1) == g.H && x2->size(2) == g.Wd, "x2 shape");
    if (g.Cin1 % 64 != 0 || x2->size(3) % 64 != 0) {
      xcat = at::cat({x, *x2}, 3);
      g.Cin1 = g.Cin = xcat.size(3);
    } else {
      g.A2 = cptr(*x2);
      g.Cin += x2->size(3);
    }
  }
  SHAI_CHECK(g.Cin % 8 == 0 && g.Cin1 % 8 == 0, "conv2d: input channels must be multiples of 8");
  g.KH = kh;
  g.KW = kw;
  g.stride = stride;
  g.pad = pad;
  g.upsample = upsample;
  const int IH = upsample ? 2 * g.H : g.H, IW = upsample ? 2 * g.Wd : g.Wd;
  SHAI_CHECK(!upsample || stride == 1, "upsample requires stride 1");
  g.OH = (IH + 2 * pad - kh) / stride + 1;
  g.OW = (IW + 2 * pad - kw) / stride + 1;
  if (up_phases) {
    // nearest-2x upsample + 3x3 pad-1 conv as 4 phase 2x2 convs over the source (w: [4 Cout, 4 Cin] phase weights,
    // ops.pack_up2_phase_weight); v4 kernel only (gemm_8ph.hip CONV 3)
    SHAI_CHECK(upsample && kh == 2 && kw == 2 && stride == 1 && pad == 0 && !x2 && !in_scale && !residual,
               "up_phases: phase weights of a plain upsample + 3x3 conv (kh = kw = 2, pad 0, no concat / norm / residual)");
    g.upsample = 2;
    g.OH = 2 * g.H;
    g.OW = 2 * g.Wd;
  }
  SHAI_CHECK(out.size(0) == g.Nimg && out.size(1) == g.OH && out.size(2) == g.OW, "conv2d out shape ", out.sizes(),
             " expected spatial ", g.OH, "x", g.OW);
  g.N = out.size(3);
  g.K = kh * kw * g.Cin;
  const int wsets = up_phases ? 4 : 1;
  SHAI_CHECK(w.size(0) == wsets * g.N && w.numel() == (long)wsets * g.N * g.K, "conv2d weight must be [Cout, KH*KW*Cin]",
             up_phases ? " per phase" : "");
  g.M = g.Nimg * g.OH * g.OW;
  g.A = xcat.defined() ? cptr(xcat) : cptr(x);
  g.W = cptr(w);
  g.C = mptr(out);
  g.lda = g.K;
  g.ldw = g.K;
  g.ldc = g.N;
  g.batch = 1;
  g.alpha = 1.f;
  g.res_alpha = res_alpha;
  g.act = act;
  if (bias) {
    check_bf16(*bias, "bias");
    g.bias = cptr(*bias);
  }
  if (bias2d) {
    check_bf16(*bias2d, "bias2d");
    SHAI_CHECK(bias2d->is_contiguous() && bias2d->size(0) == g.Nimg && bias2d->size(-1) == g.N, "bias2d [N, Cout]");
    g.bias2d = cptr(*bias2d);
    g.rows_per_bias2d = g.OH * g.OW;
  }
  if (residual) {
    check_bf16(*residual, "residual");
    SHAI_CHECK(residual->is_contiguous() && residual->numel() == (long)g.M * g.N, "residual shape");
    g.residual = cptr(*residual);
    g.ldr = g.N;
  }
  if (in_scale) {
    SHAI_CHECK(in_shift.has_value(), "in_scale requires in_shift");
    check_f32(*in_scale, "in_scale");
    check_f32(*in_shift, "in_shift");
    SHAI_CHECK(in_scale->numel() == (long)g.Nimg * g.Cin && in_shift->numel() == (long)g.Nimg * g.Cin,
               "in_scale / in_shift must be [N, Cin]");
    g.in_scale = in_scale->data_ptr<float>();
    g.in_shift = in_shift->data_ptr<float>();
    g.in_act = in_act;
  }
  OutStats st;
  attach_norm_io(g, ln_mr, ln_s, gn_part, ln_stats, ln_eps, &st);
  SHAI_CHECK(g.upsample != 2 || (shai::gemm4_supported(g) && use_v2(g, x.numel() * 2, w.numel() * 2, 0)),
             "up_phases: shape not supported by the phase conv (needs Cin % 64 == 0, H W % 256 == 0, v2 GEMM path)");
  // Halo-tiled conv (conv_halo.hip): GroupNorm(+SiLU) convs (SHAI_HALO_CONV >= 1) and, at mode 2, every 3x3
  // stride-1 conv it supports; the output's GroupNorm partials come from its epilogue.
  const int hmode = halo_conv_mode();
  if (hmode > 0 && g.row_mr == nullptr && st.ln_mr == nullptr && (g.in_scale != nullptr || hmode >= 2) &&
      shai::conv_halo_supported(g)) {
    g.col_part = st.gn_part;
    shai::launch_conv_halo(g, stream(), g_halo_waves);
    return;
  }
  Tensor xn;
  if (g.in_scale != nullptr) {
    // no fused kernel for this shape: the normalised input as one vectorised pass (fused concat read), then the
    // tuned conv on it -- never the v1 kernel's per-tap in-gather normalisation
    SHAI_CHECK(g.in_act == 0 || g.in_act == 1, "conv2d input norm activation must be none / silu");
    xn = at::empty({(long)g.Nimg, (long)g.H, (long)g.Wd, (long)g.Cin}, x.options());
    shai::GroupNormArgs a{};
    a.x = g.A;
    a.x2 = g.A2;
    a.C1 = g.A2 ? g.Cin1 : g.Cin;
    a.scale = const_cast<float*>(g.in_scale);
    a.shift = const_cast<float*>(g.in_shift);
    a.out = mptr(xn);
    a.N = g.Nimg;
    a.HW = g.H * g.Wd;
    a.C = g.Cin;
    a.silu = g.in_act == 1;
    shai::launch_groupnorm_apply(a, stream());
    g.A = cptr(xn);
    g.A2 = nullptr;
    g.Cin1 = g.Cin;
    g.in_scale = g.in_shift = nullptr;
  }
  run_gemm(g, x, xn.defined() ? xn.numel() * 2 : (xcat.defined() ? xcat.numel() * 2 : x.numel() * 2),
           w.numel() * 2, (g.A2 != nullptr) ? x2->numel() * 2 : 0, &st);
}

// ---------------------------------------------------------------- attention
void flash_attn(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o, double scale, bool causal,
                int64_t causal_offset, const optional<Tensor>& kv_lens, const optional<Tensor>& q_lens,
                const optional<Tensor>& bias, const optional<Tensor>& block_table) {
  check_rows(q, "q");
  check_rows(k, "k");
  check_rows(v, "v");
  check_rows(o, "o");
  SHAI_CHECK(q.dim() == 4 && o.dim() == 4, "q/o must be [B, S, H, D]");
  shai::AttnArgs a{};
  a.B = q.size(0);
  a.Sq = q.size(1);
  a.Hq = q.size(2);
  a.D = q.size(3);
  SHAI_CHECK(a.D == 64 || a.D == 128 || (a.D == 512 && a.Hq == 1),
             "flash_attn supports head dim 64 / 128 (and 512 with one head: the VAE mid-block), got ", a.D);
  SHAI_CHECK(q.stride(2) == a.D && o.stride(2) == a.D, "heads must be packed (head stride == D)");
  if (block_table) {
    // k/v are caches [num_blocks, Hkv, 64, D]
    SHAI_CHECK(k.dim() == 4 && k.size(2) == 64 && k.size(3) == a.D && k.is_contiguous() && v.is_contiguous(),
               "paged k/v must be [blocks, Hkv, 64, D]");
    check_i32(*block_table, "block_table");
    SHAI_CHECK(kv_lens.has_value(), "paged attention needs kv_lens");
    a.Hkv = k.size(1);
    a.block_table = block_table->data_ptr<int>();
    a.max_blocks = block_table->size(1);
    a.kc_bs = k.stride(0);
    a.kc_hs = k.stride(1);
    a.Skv = a.max_blocks * 64;
  } else {
    SHAI_CHECK(k.dim() == 4 && v.dim() == 4 && k.size(3) == a.D && k.stride(2) == a.D && v.stride(2) == a.D,
               "k/v must be [B, S, Hkv, D] with packed heads");
    a.Hkv = k.size(2);
    a.Skv = k.size(1);
    a.k_bs = k.size(0) == 1 ? 0 : k.stride(0);
    a.k_ts = k.stride(1);
    a.v_bs = v.size(0) == 1 ? 0 : v.stride(0);
    a.v_ts = v.stride(1);
  }
  SHAI_CHECK(a.Hq % a.Hkv == 0, "Hq must be a multiple of Hkv");
  a.q = cptr(q);
  a.k = cptr(k);
  a.v = cptr(v);
  a.o = mptr(o);
  a.q_bs = q.stride(0);
  a.q_ts = q.stride(1);
  a.o_bs = o.stride(0);
  a.o_ts = o.stride(1);
  a.scale = scale;
  a.causal = causal;
  a.causal_offset = causal_offset;
  if (kv_lens) {
    check_i32(*kv_lens, "kv_lens");
    a.kv_lens = kv_lens->data_ptr<int>();
  }
  if (q_lens) {
    check_i32(*q_lens, "q_lens");
    a.q_lens = q_lens->data_ptr<int>();
  }
  if (bias) {
    check_bf16(*bias, "bias");
    SHAI_CHECK(bias->is_contiguous() && bias->numel() == (long)a.Hq * a.Sq * a.Skv, "bias must be [Hq, Sq, Skv]");
    a.bias = cptr(*bias);
  }
  if (a.D == 512) {
    SHAI_CHECK(shai::attn512_supported(a), "D = 512 attention: one head, no mask / bias / causal / paged K/V, "
                                           "8-element aligned strides");
    shai::launch_attn512(a, stream());
    return;
  }
  shai::launch_flash_attn(a, stream());
}

// Packed varlen prefill attention over the paged KV cache: q / o are flat [T, Hq, D] (no padding rows);
// sequence b's queries are rows q_start[b] .. + q_lens[b] - 1, its keys the first kv_lens[b] cache entries
// of its block table; causal with offset kv_len - q_len.  max_q = max(q_lens) sizes the grid.
void paged_attn_varlen(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, const Tensor& o,
                       const Tensor& block_table, const Tensor& kv_lens, const Tensor& q_lens, const Tensor& q_start,
                       int64_t max_q, double scale, bool causal) {
  check_rows(q, "q");
  check_rows(o, "o");
  SHAI_CHECK(q.dim() == 3 && o.dim() == 3 && q.sizes() == o.sizes(), "q/o must be [T, H, D]");
  check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  check_i32(block_table, "block_table");
  check_i32(kv_lens, "kv_lens");
  check_i32(q_lens, "q_lens");
  check_i32(q_start, "q_start");
  shai::AttnArgs a{};
  a.B = block_table.size(0);
  SHAI_CHECK(kv_lens.numel() == a.B && q_lens.numel() == a.B && q_start.numel() == a.B, "per-sequence [B] metadata");
  SHAI_CHECK(max_q >= 1, "max_q >= 1");
  a.Sq = (int)max_q;
  a.Hq = q.size(1);
  a.D = q.size(2);
  SHAI_CHECK(a.D == 64 || a.D == 128, "paged_attn_varlen supports head dim 64 / 128, got ", a.D);
  SHAI_CHECK(q.stride(1) == a.D && o.stride(1) == a.D, "heads must be packed (head stride == D)");
  SHAI_CHECK(k_cache.dim() == 4 && k_cache.size(2) == 64 && k_cache.size(3) == a.D && k_cache.is_contiguous() &&
                 v_cache.is_contiguous() && v_cache.sizes() == k_cache.sizes(),
             "paged k/v must be [blocks, Hkv, 64, D]");
  a.Hkv = k_cache.size(1);
  SHAI_CHECK(a.Hq % a.Hkv == 0, "Hq must be a multiple of Hkv");
  a.block_table = block_table.data_ptr<int>();
  a.max_blocks = block_table.size(1);
  a.kc_bs = k_cache.stride(0);
  a.kc_hs = k_cache.stride(1);
  a.Skv = a.max_blocks * 64;
  a.q = cptr(q);
  a.k = cptr(k_cache);
  a.v = cptr(v_cache);
  a.o = mptr(o);
  a.q_ts = q.stride(0);
  a.o_ts = o.stride(0);
  a.scale = scale;
  a.causal = causal;
  a.kv_lens = kv_lens.data_ptr<int>();
  a.q_lens = q_lens.data_ptr<int>();
  a.q_start = q_start.data_ptr<int>();
  shai::launch_flash_attn(a, stream());
}

void decode_attn(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, const Tensor& o,
                 const Tensor& block_table, const Tensor& ctx_lens, const Tensor& ws, int64_t num_splits,
                 double scale) {
  check_rows(q, "q");
  check_rows(o, "o");
  check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  check_i32(block_table, "block_table");
  check_i32(ctx_lens, "ctx_lens");
  check_f32(ws, "ws");
  SHAI_CHECK(q.dim() == 3 && k_cache.dim() == 4 && k_cache.size(2) == 64, "decode_attn shapes");
  shai::DecodeAttnArgs a{};
  a.B = q.size(0);
  a.Hq = q.size(1);
  a.D = q.size(2);
  a.Hkv = k_cache.size(1);
  SHAI_CHECK(a.D == 64 || a.D == 128, "decode_attn head dim 64/128");
  SHAI_CHECK(a.Hq % a.Hkv == 0 && a.Hq / a.Hkv <= 8, "decode_attn GQA group must be <= 8");
  SHAI_CHECK(q.stride(1) == a.D && o.stride(1) == a.D, "packed heads");
  a.q = cptr(q);
  a.o = mptr(o);
  a.k_cache = cptr(k_cache);
  a.v_cache = cptr(v_cache);
  a.block_table = block_table.data_ptr<int>();
  a.ctx_lens = ctx_lens.data_ptr<int>();
  a.max_blocks = block_table.size(1);
  a.num_splits = num_splits;
  a.ws = ws.data_ptr<float>();
  SHAI_CHECK(ws.numel() * 4 >= (long)shai::decode_attn_workspace(a.B, a.Hq, a.D, num_splits), "ws too small");
  a.q_bs = q.stride(0);
  a.o_bs = o.stride(0);
  a.scale = scale;
  shai::launch_decode_attn(a, stream());
}

// Fused decode step on the packed QKV rows [B, (h + 2 hk) D]: RoPE on q and k, this step's k / v into the paged
// cache at slots, attention over the cached context plus the new token (replaces rope_qkv_cache +
// decode_attn in the decode graph).
// Decode QKV projection with a folded RMSNorm, left as split-K partials for decode_attn_rope to fold (one launch
// fewer per layer): the skinny kernel with the tuned K-group count (at least 2), no fold launch.  Returns the fp32
// workspace [kg][M][N] partials followed by [kg][M] row sums of squares; kg = numel / (M (N + 1)).
Tensor gemm_partials(const Tensor& a, const Tensor& w, double rms_eps) {
  check_rows(a, "a");
  check_rows(w, "w");
  SHAI_CHECK(a.dim() == 2 && w.dim() == 2 && a.size(1) == w.size(1) && rms_eps >= 0, "gemm_partials: a [M, K], w [N, K]");
  shai::GemmArgs g{};
  g.A = cptr(a);
  g.W = cptr(w);
  g.M = a.size(0);
  g.K = a.size(1);
  g.N = w.size(0);
  g.lda = a.stride(0);
  g.ldw = w.stride(0);
  g.ldc = g.N;
  g.batch = 1;
  g.alpha = 1.0;
  g.res_alpha = 1.0;
  g.rms = 1;
  g.rms_eps = (float)rms_eps;
  SHAI_CHECK(g.K % 8 == 0 && shai::skinny_supported(g), "gemm_partials: problem not supported by the skinny kernel");
  Choice c{-1, 1};
  int kg = (lookup_choice(g, gemm_key(g), &c) && (c.cfg == kSkinnyCfg || c.cfg == kSkinnyFixCfg)) ? c.splits
                                                                                                : shai::skinny_kgroups(g);
  static const int env_kg = [] {  // A/B knob: pin the K-group count of the partials
    const char* e = getenv("SHAI_QKV_PART_KG");
    return e ? atoi(e) : 0;
  }();
  if (env_kg > 0) kg = env_kg;
  kg = std::min(std::max(kg, 2), shai::skinny_max_kgroups(g));
  SHAI_CHECK(kg >= 2, "gemm_partials: K too small for split-K");
  Tensor ws = at::empty({(long)kg * g.M * (g.N + 1)}, a.options().dtype(at::kFloat));
  g.C = nullptr;  // partials only: nothing is written to C
  shai::launch_skinny_kg(g, ws.data_ptr<float>(), kg, stream(), false, false);
  return ws;
}

void decode_attn_rope(const Tensor& qkv, const Tensor& k_cache, const Tensor& v_cache, const Tensor& o,
                      const Tensor& block_table, const Tensor& ctx_lens, const Tensor& positions, const Tensor& cos,
                      const Tensor& sin, const Tensor& slots, const Tensor& ws, int64_t h, int64_t hk,
                      int64_t num_splits, double scale, const optional<Tensor>& qkv_ws, int64_t qkv_kg,
                      int64_t qkv_k, double qkv_eps) {
  const bool part = qkv_ws.has_value();
  if (!part) check_bf16(qkv, "qkv");  // partials path: qkv is a placeholder (the partials), never read
  check_rows(o, "o");
  check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  check_i32(block_table, "block_table");
  check_i32(ctx_lens, "ctx_lens");
  check_i32(positions, "positions");
  check_i32(slots, "slots");
  check_f32(ws, "ws");
  SHAI_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat && cos.is_contiguous() &&
                 sin.is_contiguous(), "rope tables: contiguous fp32");
  SHAI_CHECK(k_cache.dim() == 4 && k_cache.size(2) == 64 && k_cache.size(1) == hk, "decode_attn_rope cache shape");
  shai::DecodeAttnArgs a{};
  a.D = k_cache.size(3);
  a.B = part ? o.size(0) : qkv.size(0);
  a.Hq = h;
  a.Hkv = hk;
  SHAI_CHECK(a.D == 64 || a.D == 128, "decode_attn head dim 64/128");
  SHAI_CHECK(a.Hq % a.Hkv == 0 && a.Hq / a.Hkv <= 8, "decode_attn GQA group must be <= 8");
  if (part) {  // q / k / v come from the QKV GEMM's split-K partials (gemm_partials); qkv is not read
    check_f32(*qkv_ws, "qkv_ws");
    const long n = (h + 2 * hk) * a.D;
    SHAI_CHECK(qkv_kg >= 2 && qkv_k > 0 && qkv_eps >= 0 &&
                   qkv_ws->numel() == qkv_kg * (long)a.B * (n + 1),
               "qkv_ws must be the [kg][B][(h + 2 hk) D] partials + [kg][B] row sums of gemm_partials");
    a.qkv_ws = qkv_ws->data_ptr<float>();
    a.qkv_kg = qkv_kg;
    a.qkv_n = n;
    a.qkv_k = qkv_k;
    a.qkv_eps = qkv_eps;
  } else {
    SHAI_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1 && qkv.size(1) >= (h + 2 * hk) * a.D, "qkv rows");
  }
  SHAI_CHECK(o.dim() == 2 && o.size(0) == a.B && o.size(1) == h * a.D && o.stride(1) == 1, "o [B, h D]");
  SHAI_CHECK(cos.size(1) == a.D / 2 && sin.sizes() == cos.sizes(), "rope tables [max_pos, D / 2]");
  SHAI_CHECK(positions.numel() >= a.B && slots.numel() >= a.B && ctx_lens.numel() >= a.B, "per-row inputs");
  if (part) {
    // q / k / v come from the partials; knew != nullptr only selects the fused RoPE / KV-write path
    const shai::bf16_t* flag = reinterpret_cast<const shai::bf16_t*>(a.qkv_ws);
    a.q = a.knew = a.vnew = flag;
    a.q_bs = a.new_bs = 0;
  } else {
    const shai::bf16_t* base = cptr(qkv);
    a.q = base;
    a.knew = base + h * a.D;
    a.vnew = base + (h + hk) * a.D;
    a.q_bs = a.new_bs = qkv.stride(0);
  }
  a.o = mptr(o);
  a.o_bs = o.stride(0);
  a.k_cache = cptr(k_cache);
  a.v_cache = cptr(v_cache);
  a.block_table = block_table.data_ptr<int>();
  a.ctx_lens = ctx_lens.data_ptr<int>();
  a.positions = positions.data_ptr<int>();
  a.slots = slots.data_ptr<int>();
  a.rope_cos = cos.data_ptr<float>();
  a.rope_sin = sin.data_ptr<float>();
  a.max_blocks = block_table.size(1);
  a.num_splits = num_splits;
  a.ws = ws.data_ptr<float>();
  SHAI_CHECK(ws.numel() * 4 >= (long)shai::decode_attn_workspace(a.B, a.Hq, a.D, num_splits), "ws too small");
  a.scale = scale;
  shai::launch_decode_attn(a, stream());
}

void kv_write(const Tensor& k, const Tensor& v, const Tensor& k_cache, const Tensor& v_cache, const Tensor& slots) {
  check_rows(k, "k");
  check_rows(v, "v");
  check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  check_i32(slots, "slots");
  SHAI_CHECK(k.dim() == 3 && k_cache.dim() == 4, "k [T, Hkv, D], cache [blocks, Hkv, 64, D]");
  SHAI_CHECK(k.stride(1) == k.size(2) && v.stride(1) == v.size(2), "packed heads");
  shai::launch_kv_write(cptr(k), cptr(v), mptr(k_cache), mptr(v_cache), slots.data_ptr<int>(), k.size(0), k.size(1),
                        k.size(2), k.stride(0), v.stride(0), stream());
}

// ---------------------------------------------------------------- elementwise
void gated_act(const Tensor& x, const Tensor& out, int64_t act, bool gate_first) {
  check_rows(x, "x");
  check_bf16(out, "out");
  SHAI_CHECK(out.is_contiguous(), "out contiguous");
  const int F = out.size(-1);
  SHAI_CHECK(x.size(-1) == 2 * F && F % 8 == 0, "gated_act: x last dim must be 2*F, F % 8 == 0");
  const long rows = out.numel() / F;
  const long xs = x.dim() >= 2 ? x.stride(-2) : 2 * F;
  SHAI_CHECK(x.dim() == 2 || x.is_contiguous(), "gated_act x must be 2D strided or contiguous");
  shai::launch_gated_act(cptr(x), mptr(out), rows, F, xs, act, gate_first, stream());
}

// A non-owning device tensor over memory this library did not allocate through torch (the xGMI P2P staging slot:
// IPC-exported uncached memory a row-parallel GEMM writes its partial product into).  The caller keeps the
// memory alive for the tensor's lifetime.
Tensor from_ptr(int64_t ptr, at::IntArrayRef size, at::ScalarType dtype, int64_t device) {
  SHAI_CHECK(ptr != 0 && (ptr & 15) == 0, "from_ptr: null or misaligned pointer");
  return at::from_blob(reinterpret_cast<void*>(ptr), size,
                       at::TensorOptions().dtype(dtype).device(at::kCUDA, (c10::DeviceIndex)device));
}

void bias_act(const Tensor& x, const optional<Tensor>& bias, const optional<Tensor>& residual, const Tensor& out,
              int64_t act, double alpha) {
  check_bf16(x, "x");
  check_bf16(out, "out");
  SHAI_CHECK(x.is_contiguous() && out.is_contiguous(), "bias_act contiguous");
  const int D = x.size(-1);
  SHAI_CHECK(D % 8 == 0, "D % 8");
  if (residual) SHAI_CHECK(residual->is_contiguous() && residual->numel() == x.numel(), "residual");
  shai::launch_bias_act(cptr(x), optr(bias), optr(residual), mptr(out), x.numel() / D, D, act, alpha, stream());
}

void rope(const Tensor& x, const Tensor& positions, const Tensor& cos, const Tensor& sin, int64_t rot_dim, bool neox) {
  check_bf16(x, "x");
  check_i32(positions, "positions");
  check_f32(cos, "cos");
  check_f32(sin, "sin");
  SHAI_CHECK(x.dim() == 3 && x.stride(1) == x.size(2), "rope x must be [T, H, Dh] with packed heads");
  shai::launch_rope(mptr(x), positions.data_ptr<int>(), cos.data_ptr<float>(), sin.data_ptr<float>(), x.size(0),
                    x.size(1), x.size(2), rot_dim, x.stride(0), neox, stream());
}

void rope_qkv_cache(const Tensor& qkv, const Tensor& positions, const Tensor& cos, const Tensor& sin,
                    const Tensor& k_cache, const Tensor& v_cache, const Tensor& slots, int64_t H, int64_t Hkv) {
  check_bf16(qkv, "qkv");
  check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  check_i32(positions, "positions");
  check_i32(slots, "slots");
  check_f32(cos, "cos");
  check_f32(sin, "sin");
  SHAI_CHECK(qkv.dim() == 2 && qkv.stride(0) % 8 == 0, "qkv must be [T, (H + 2Hkv) * D] with 16B-aligned rows");
  SHAI_CHECK(k_cache.dim() == 4 && k_cache.is_contiguous() && v_cache.is_contiguous() && k_cache.size(1) == Hkv &&
                 k_cache.size(2) == 64,
             "caches must be contiguous [blocks, Hkv, 64, D]");
  const int D = k_cache.size(3);
  SHAI_CHECK(D % 16 == 0 && qkv.size(1) == (H + 2 * Hkv) * D, "qkv width / head dim mismatch");
  SHAI_CHECK(cos.size(-1) == D / 2, "cos/sin must be [max_pos, D/2] (full-dim NeoX rotation)");
  const int T = qkv.size(0);
  SHAI_CHECK(positions.numel() == T && slots.numel() == T, "positions / slots must have T entries");
  shai::launch_rope_qkv_cache(mptr(qkv), qkv.stride(0), positions.data_ptr<int>(), cos.data_ptr<float>(),
                              sin.data_ptr<float>(), mptr(k_cache), mptr(v_cache), slots.data_ptr<int>(), T, H, Hkv,
                              D, stream());
}

void sample(const Tensor& logits, const Tensor& temps, const Tensor& top_k, const Tensor& top_p,
            const Tensor& uniforms, const Tensor& out) {
  SHAI_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1, "logits must be a 2D GPU tensor");
  const bool bf16 = logits.scalar_type() == at::kBFloat16;
  SHAI_CHECK(bf16 || logits.scalar_type() == at::kFloat, "logits must be bf16 or fp32");
  const int B = logits.size(0);
  check_f32(temps, "temps");
  check_f32(top_p, "top_p");
  check_f32(uniforms, "uniforms");
  check_i32(top_k, "top_k");
  check_i32(out, "out");
  SHAI_CHECK(temps.numel() == B && top_p.numel() == B && uniforms.numel() == B && top_k.numel() == B &&
                 out.numel() == B,
             "per-row parameter sizes");
  shai::launch_sample(logits.data_ptr(), bf16, logits.stride(0), B, logits.size(1), temps.data_ptr<float>(),
                      top_k.data_ptr<int>(), top_p.data_ptr<float>(), uniforms.data_ptr<float>(),
                      out.data_ptr<int>(), stream());
}

void rope_pairs(const Tensor& x, const Tensor& cos, const Tensor& sin) {
  check_bf16(x, "x");
  check_f32(cos, "cos");
  check_f32(sin, "sin");
  SHAI_CHECK(x.dim() == 4 && x.stride(2) == x.size(3) && x.size(3) % 8 == 0, "rope_pairs x [B, T, H, Dh]");
  SHAI_CHECK(cos.numel() == x.size(1) * x.size(3) / 2, "cos/sin must be [T, Dh/2]");
  shai::launch_rope_pairs(mptr(x), cos.data_ptr<float>(), sin.data_ptr<float>(), x.size(0), x.size(1), x.size(2),
                          x.size(3), x.stride(0), x.stride(1), stream());
}

void sched_step(const Tensor& model_out, const Tensor& latents, bool cfg, double guidance, int64_t pred_type,
                double a_t, double a_prev, double dt) {
  check_bf16(model_out, "model_out");
  check_bf16(latents, "latents");
  SHAI_CHECK(model_out.is_contiguous() && latents.is_contiguous(), "sched_step contiguous");
  const long n = latents.numel();
  SHAI_CHECK(n % 8 == 0 && model_out.numel() == (cfg ? 2 * n : n), "sched_step sizes");
  shai::launch_sched_step(cptr(model_out), mptr(latents), n, cfg, guidance, pred_type, a_t, a_prev, dt, stream());
}

// step-level batching: every image row of `latents` [B, ...] at its own step; rows_params fp32 [B, 3] =
// (a_t, a_prev, dt) per row, a_t < 0 = idle row (untouched)
void sched_step_rows(const Tensor& model_out, const Tensor& latents, bool cfg, double guidance, int64_t pred_type,
                     const Tensor& rows_params) {
  check_bf16(model_out, "model_out");
  check_bf16(latents, "latents");
  check_f32(rows_params, "rows_params");
  SHAI_CHECK(model_out.is_contiguous() && latents.is_contiguous() && rows_params.is_contiguous(),
             "sched_step_rows contiguous");
  const long n = latents.numel();
  const long B = latents.size(0);
  SHAI_CHECK(B > 0 && n % B == 0 && (n / B) % 8 == 0 && model_out.numel() == (cfg ? 2 * n : n) &&
                 rows_params.numel() == 3 * B,
             "sched_step_rows sizes");
  shai::launch_sched_step_rows(cptr(model_out), mptr(latents), n, n / B, cfg, guidance, pred_type,
                               rows_params.data_ptr<float>(), stream());
}

void softmax_(const Tensor& x, double scale) {
  check_bf16(x, "x");
  SHAI_CHECK(x.is_contiguous() && x.size(-1) % 8 == 0, "softmax contiguous, D % 8");
  shai::launch_softmax(mptr(x), x.numel() / x.size(-1), x.size(-1), scale, stream());
}

std::vector<std::string> gemm_tuning() { return gemm_tuning_table(); }

// Export / import the autotuner cache ("key=cfg,splits") so later processes skip tuning.
std::vector<std::string> gemm_tuning_export() {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  std::vector<std::string> out;
  for (auto& kv : g_tuned) out.push_back(kv.first + "=" + std::to_string(kv.second.cfg) + "," + std::to_string(kv.second.splits));
  return out;
}

int64_t gemm_tuning_import(const std::vector<std::string>& entries) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  int64_t n = 0;
  for (const auto& e : entries) {
    const auto eq = e.rfind('=');
    const auto cm = e.rfind(',');
    if (eq == std::string::npos || cm == std::string::npos || cm < eq) continue;
    const int cfg = atoi(e.substr(eq + 1, cm - eq - 1).c_str());
    const int sp = atoi(e.substr(cm + 1).c_str());
    if ((cfg < 0 || cfg >= shai::gemm2_num_cfgs()) && !is_skinny(cfg) && cfg != kLibCfg) continue;
    if (cfg == kLibCfg && !lib_enabled()) continue;
    if (sp < 1) continue;
    g_tuned[e.substr(0, eq)] = Choice{cfg, sp};
    ++n;
  }
  return n;
}

void token_feedback(const Tensor& ids, const Tensor& rowmap, const Tensor& prev) {
  SHAI_CHECK(ids.scalar_type() == at::kInt && rowmap.scalar_type() == at::kInt && prev.scalar_type() == at::kInt &&
                 ids.is_contiguous() && rowmap.is_contiguous() && prev.is_contiguous() && rowmap.numel() == ids.numel(),
             "token_feedback: int32 contiguous ids / rowmap of one length");
  shai::launch_token_feedback(ids.data_ptr<int>(), rowmap.data_ptr<int>(), prev.data_ptr<int>(), (int)ids.numel(),
                              stream());
}

void embedding(const Tensor& ids, const Tensor& table, const Tensor& out) {
  check_i32(ids, "ids");
  check_bf16(table, "table");
  check_bf16(out, "out");
  SHAI_CHECK(table.is_contiguous() && out.is_contiguous() && table.size(1) % 8 == 0, "embedding shapes");
  shai::launch_embedding(ids.data_ptr<int>(), cptr(table), mptr(out), ids.numel(), table.size(1), stream());
}

}  // namespace

void dequant_fp8(const Tensor& w8, const Tensor& scale, const Tensor& out) {
  SHAI_CHECK(w8.is_cuda() && w8.scalar_type() == at::kFloat8_e4m3fn && w8.dim() == 2 && w8.is_contiguous() &&
                 w8.size(1) % 8 == 0,
             "dequant_fp8: w8 must be a contiguous float8_e4m3fn [N, K], K % 8 == 0");
  check_f32(scale, "scale");
  check_bf16(out, "out");
  SHAI_CHECK(scale.numel() == w8.size(0) && out.is_contiguous() && out.numel() == w8.numel(), "dequant_fp8 shapes");
  shai::launch_dequant_fp8_rows(reinterpret_cast<const uint8_t*>(w8.data_ptr()), scale.data_ptr<float>(), mptr(out),
                                w8.size(0), w8.size(1), stream());
}

// y = a w^T + bias + res_alpha residual into c, and LayerNorm(y) gamma + beta into c2, on the W-stationary kernel
// (gemm_ws.hip: K = 320, N = 320, the row moments from the epilogue's registers).  Returns false (nothing launched)
// when the problem is outside the kernel's contract; the caller then runs the GEMM and the norm separately.
bool gemm_lnout(const Tensor& a, const Tensor& w, const Tensor& c, const Tensor& c2, const optional<Tensor>& bias,
                const Tensor& residual, double res_alpha, const optional<Tensor>& gamma, const optional<Tensor>& beta,
                double eps) {
  check_rows(a, "a");
  check_rows(w, "w");
  check_bf16(c, "c");
  check_bf16(c2, "c2");
  check_rows(residual, "residual");
  if (a.dim() != 2 || w.dim() != 2 || c.dim() != 2 || c2.dim() != 2 || residual.dim() != 2) return false;
  shai::GemmArgs g{};
  g.A = cptr(a);
  g.W = cptr(w);
  g.C = mptr(c);
  g.M = a.size(0);
  g.K = a.size(1);
  g.N = w.size(0);
  SHAI_CHECK(w.size(1) == g.K, "gemm_lnout K mismatch");
  SHAI_CHECK(c.size(0) == g.M && c.size(1) == g.N && c2.sizes() == c.sizes() && residual.sizes() == c.sizes(),
             "gemm_lnout output / residual shape mismatch");
  if (c.stride(0) != c2.stride(0)) return false;
  g.lda = a.stride(0);
  g.ldw = w.stride(0);
  g.ldc = c.stride(0);
  g.residual = cptr(residual);
  g.ldr = residual.stride(0);
  g.alpha = 1.f;
  g.res_alpha = (float)res_alpha;
  g.batch = 1;
  g.rows_per_bias2d = 1;
  g.rows_per_gate = 1;
  if (bias.has_value()) {
    check_bf16(*bias, "bias");
    SHAI_CHECK(bias->numel() == g.N, "gemm_lnout bias [N]");
    g.bias = cptr(*bias);
  }
  for (const optional<Tensor>* t : {&gamma, &beta})
    if (t->has_value()) {
      check_bf16(**t, "gamma/beta");
      SHAI_CHECK((*t)->numel() == g.N, "gemm_lnout gamma / beta [N]");
    }
  if (!shai::gemm_ws_lnout_supported(g)) return false;
  shai::launch_gemm_ws_lnout(g, mptr(c2), optr(gamma), optr(beta), (float)eps, stream());
  return true;
}

// W8A8 fp8 GEMM (gemm_f8.hip): a8 [M, K] / w8 [N, K] float8_e4m3fn, a_scale [M] / w_scale [N] fp32.
// cfg < 0 picks the tile: 256 x 128 when that still yields >= 256 tiles, else 128 x 128.
void gemm_f8(const Tensor& a8, const Tensor& w8, const Tensor& a_scale, const Tensor& w_scale, const Tensor& c,
             const optional<Tensor>& bias, const optional<Tensor>& residual, double res_alpha, int64_t act, bool glu,
             int64_t cfg) {
  SHAI_CHECK(a8.is_cuda() && a8.scalar_type() == at::kFloat8_e4m3fn && a8.dim() == 2 && a8.stride(1) == 1,
             "gemm_f8: a8 must be float8_e4m3fn [M, K] with unit column stride");
  SHAI_CHECK(w8.is_cuda() && w8.scalar_type() == at::kFloat8_e4m3fn && w8.dim() == 2 && w8.is_contiguous(),
             "gemm_f8: w8 must be a contiguous float8_e4m3fn [N, K]");
  check_f32(a_scale, "a_scale");
  check_f32(w_scale, "w_scale");
  check_bf16(c, "c");
  const long M = a8.size(0), K = a8.size(1), N = w8.size(0);
  SHAI_CHECK(w8.size(1) == K && a_scale.numel() == M && w_scale.numel() == N, "gemm_f8 shapes");
  SHAI_CHECK(c.dim() == 2 && c.size(0) == M && c.size(1) == (glu ? N / 2 : N) && c.stride(1) == 1, "gemm_f8: c shape");
  shai::GemmArgs g{};
  g.M = (int)M;
  g.N = (int)N;
  g.K = (int)K;
  g.lda = a8.stride(0);
  g.ldw = K;
  g.C = mptr(c);
  g.ldc = c.stride(0);
  g.alpha = 1.f;
  g.res_alpha = (float)res_alpha;
  g.act = (int)act;
  g.glu = glu ? 1 : 0;
  g.batch = 1;
  if (bias.has_value()) {
    check_bf16(*bias, "bias");
    SHAI_CHECK(bias->numel() == N, "gemm_f8: bias [N]");
    g.bias = cptr(*bias);
  }
  if (residual.has_value()) {
    check_bf16(*residual, "residual");
    SHAI_CHECK(residual->dim() == 2 && residual->size(0) == M && residual->size(1) == c.size(1) &&
                   residual->stride(1) == 1, "gemm_f8: residual shape");
    g.residual = cptr(*residual);
    g.ldr = residual->stride(0);
  }
  SHAI_CHECK(shai::gemm_f8_supported(g), "gemm_f8: unsupported problem (K, lda multiples of 16; GLU needs N % 4 == 0)");
  if (cfg < 0) cfg = ((M + 255) / 256) * ((N + 127) / 128) >= 256 ? 0 : 1;
  shai::launch_gemm_f8(g, reinterpret_cast<const uint8_t*>(a8.data_ptr()), reinterpret_cast<const uint8_t*>(w8.data_ptr()),
                       a_scale.data_ptr<float>(), w_scale.data_ptr<float>(), (int)cfg, stream());
}

void quant_rows_fp8(const Tensor& x, const Tensor& out, const Tensor& scale, double rms_eps) {
  check_bf16(x, "x");
  SHAI_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "quant_rows_fp8: x [M, K], 16-B aligned rows");
  SHAI_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat8_e4m3fn && out.dim() == 2 && out.stride(1) == 1 &&
                 out.size(0) == x.size(0) && out.size(1) == x.size(1) && out.stride(0) % 8 == 0,
             "quant_rows_fp8: out float8_e4m3fn [M, K]");
  check_f32(scale, "scale");
  SHAI_CHECK(scale.numel() == x.size(0), "quant_rows_fp8: scale [M]");
  SHAI_CHECK(shai::quant_rows_fp8_supported((int)x.size(1)), "quant_rows_fp8: K % 8 == 0");
  if (x.size(0) == 0) return;
  shai::launch_quant_rows_fp8(cptr(x), x.stride(0), (int)x.size(0), (int)x.size(1),
                              reinterpret_cast<uint8_t*>(out.data_ptr()), out.stride(0), scale.data_ptr<float>(),
                              (float)rms_eps, stream());
}

TORCH_LIBRARY(shai, m) {
  m.def("from_ptr(int ptr, int[] size, ScalarType dtype, int device) -> Tensor", &from_ptr);
  m.def("gemm_f8(Tensor a8, Tensor w8, Tensor a_scale, Tensor w_scale, Tensor(a!) c, Tensor? bias, Tensor? residual, float res_alpha, int act, bool glu, int cfg=-1) -> ()");
  m.def("quant_rows_fp8(Tensor x, Tensor(a!) out, Tensor(b!) scale, float rms_eps) -> ()");
  m.def("rmsnorm(Tensor x, Tensor? w, Tensor(a!) out, Tensor? residual, Tensor(b!)? residual_out, float eps, float w_offset) -> ()");
  m.def("layernorm(Tensor x, Tensor? w, Tensor? b, Tensor(a!) out, Tensor? residual, Tensor(b!)? residual_out, float eps) -> ()");
  m.def("groupnorm_stats(Tensor x, Tensor? x2, Tensor? gamma, Tensor? beta, Tensor(a!) partials, Tensor(b!) scale, Tensor(c!) shift, Tensor(d!)? counters, int G, float eps) -> ()");
  m.def("groupnorm_apply(Tensor x, Tensor? x2, Tensor scale, Tensor shift, Tensor(a!) out, bool silu) -> ()");
  m.def("groupnorm_from_partials(Tensor part1, Tensor? part2, int C1, int C2, int Nimg, int HW, Tensor? gamma, Tensor? beta, Tensor(a!) scale, Tensor(b!) shift, int G, float eps) -> ()");
  m.def("col_partials(Tensor x, Tensor(a!) part) -> ()");
  m.def("row_moments(Tensor x, Tensor(a!) mr, float eps) -> ()");
  m.def("gemm(Tensor a, Tensor w, Tensor(a!) c, Tensor? bias, Tensor? bias2d, int rows_per_bias2d, Tensor? residual, float alpha, float res_alpha, int act, bool glu, Tensor? gate=None, int rows_per_gate=1, int force_cfg=-1, float rms_eps=-1.0, Tensor? w_scale=None, Tensor? ln_mr=None, Tensor? ln_s=None, Tensor(b!)? gn_part=None, Tensor(c!)? ln_stats=None, float ln_eps=1e-5, int w_slice_rows=0) -> ()");
  m.def("dequant_fp8(Tensor w8, Tensor scale, Tensor(a!) out) -> ()");
  m.def("layernorm_mod(Tensor x, Tensor scale, Tensor shift, Tensor(a!) out, int rows_per_mod, float eps) -> ()");
  m.def("qk_norm_rope(Tensor(a!) x, Tensor? q_w, Tensor? k_w, Tensor? cos, Tensor? sin, int H, int D, int S, float eps) -> ()");
  m.def("conv2d(Tensor x, Tensor? x2, Tensor w, Tensor(a!) out, Tensor? bias, Tensor? bias2d, Tensor? residual, Tensor? in_scale, Tensor? in_shift, int in_act, int kh, int kw, int stride, int pad, bool upsample, int act, float res_alpha, Tensor? ln_mr=None, Tensor? ln_s=None, Tensor(b!)? gn_part=None, Tensor(c!)? ln_stats=None, float ln_eps=1e-5, bool up_phases=False) -> ()");
  m.def("flash_attn(Tensor q, Tensor k, Tensor v, Tensor(a!) o, float scale, bool causal, int causal_offset, Tensor? kv_lens, Tensor? q_lens, Tensor? bias, Tensor? block_table) -> ()");
  m.def("paged_attn_varlen(Tensor q, Tensor k_cache, Tensor v_cache, Tensor(a!) o, Tensor block_table, Tensor kv_lens, Tensor q_lens, Tensor q_start, int max_q, float scale, bool causal) -> ()");
  m.def("decode_attn(Tensor q, Tensor k_cache, Tensor v_cache, Tensor(a!) o, Tensor block_table, Tensor ctx_lens, Tensor(b!) ws, int num_splits, float scale) -> ()");
  m.def("kv_write(Tensor k, Tensor v, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor slots) -> ()");
  m.def("gated_act(Tensor x, Tensor(a!) out, int act, bool gate_first) -> ()");
  m.def("bias_act(Tensor x, Tensor? bias, Tensor? residual, Tensor(a!) out, int act, float alpha) -> ()");
  m.def("rope(Tensor(a!) x, Tensor positions, Tensor cos, Tensor sin, int rot_dim, bool neox) -> ()");
  m.def("rope_pairs(Tensor(a!) x, Tensor cos, Tensor sin) -> ()");
  m.def("sample(Tensor logits, Tensor temps, Tensor top_k, Tensor top_p, Tensor uniforms, Tensor(a!) out) -> ()");
  m.def("rope_qkv_cache(Tensor(a!) qkv, Tensor positions, Tensor cos, Tensor sin, Tensor(b!) k_cache, Tensor(c!) v_cache, Tensor slots, int H, int Hkv) -> ()");
  m.def("sched_step(Tensor model_out, Tensor(a!) latents, bool cfg, float guidance, int pred_type, float a_t, float a_prev, float dt) -> ()");
  m.def("sched_step_rows(Tensor model_out, Tensor(a!) latents, bool cfg, float guidance, int pred_type, Tensor rows_params) -> ()");
  m.def("softmax_(Tensor(a!) x, float scale) -> ()");
  m.def("embedding(Tensor ids, Tensor table, Tensor(a!) out) -> ()");
  m.def("token_feedback(Tensor(a!) ids, Tensor rowmap, Tensor prev) -> ()");
  m.def("decode_attn_rope(Tensor qkv, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor(c!) o, Tensor block_table, "
        "Tensor ctx_lens, Tensor positions, Tensor cos, Tensor sin, Tensor slots, Tensor(d!) ws, int h, int hk, "
        "int num_splits, float scale, Tensor? qkv_ws=None, int qkv_kg=0, int qkv_k=0, float qkv_eps=-1.0) -> ()");
  m.def("gemm_partials(Tensor a, Tensor w, float rms_eps) -> Tensor");
  m.def("gemm_lnout(Tensor a, Tensor w, Tensor(a!) c, Tensor(b!) c2, Tensor? bias, Tensor residual, float res_alpha, Tensor? gamma, Tensor? beta, float eps) -> bool");
  m.def("gemm_tuning() -> str[]", &gemm_tuning);
  m.def("gemm_tuning_export() -> str[]", &gemm_tuning_export);
  m.def("gemm_tuning_import(str[] entries) -> int", &gemm_tuning_import);
  m.def("set_halo_conv(int mode, int waves=-1) -> int", &set_halo_conv);
  m.def("set_flash128x2(int mode) -> int", [](int64_t mode) -> int64_t { return shai::set_flash128x2((int)mode); });
  m.def("set_decode_wb(int mode) -> int", [](int64_t mode) -> int64_t { return shai::set_decode_wb((int)mode); });
}

TORCH_LIBRARY_IMPL(shai, CUDA, m) {
  m.impl("rmsnorm", &rmsnorm);
  m.impl("layernorm", &layernorm);
  m.impl("groupnorm_stats", &groupnorm_stats);
  m.impl("groupnorm_from_partials", &groupnorm_from_partials);
  m.impl("col_partials", &col_partials);
  m.impl("row_moments", &row_moments);
  m.impl("groupnorm_apply", &groupnorm_apply);
  m.impl("gemm", &gemm);
  m.impl("dequant_fp8", &dequant_fp8);
  m.impl("gemm_f8", &gemm_f8);
  m.impl("gemm_lnout", &gemm_lnout);
  m.impl("quant_rows_fp8", &quant_rows_fp8);
  m.impl("layernorm_mod", &layernorm_mod);
  m.impl("qk_norm_rope", &qk_norm_rope);
  m.impl("conv2d", &conv2d);
  m.impl("flash_attn", &flash_attn);
  m.impl("paged_attn_varlen", &paged_attn_varlen);
  m.impl("decode_attn", &decode_attn);
  m.impl("kv_write", &kv_write);
  m.impl("gated_act", &gated_act);
  m.impl("bias_act", &bias_act);
  m.impl("rope", &rope);
  m.impl("rope_pairs", &rope_pairs);
  m.impl("sample", &sample);
  m.impl("rope_qkv_cache", &rope_qkv_cache);
  m.impl("sched_step", &sched_step);
  m.impl("sched_step_rows", &sched_step_rows);
  m.impl("softmax_", &softmax_);
  m.impl("embedding", &embedding);
  m.impl("token_feedback", &token_feedback);
  m.impl("decode_attn_rope", &decode_attn_rope);
  m.impl("gemm_partials", &gemm_partials);
}
