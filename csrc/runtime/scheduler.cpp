// Continuous-batching scheduler helpers (host C++, C ABI).
//
// * shai_sched_admit: FCFS admission of waiting prompts into the running set
//   under three budgets -- free KV blocks (keeping a watermark for the decode
//   growth of already-running sequences), max concurrent sequences, and a
//   per-step prefill token budget (long prompts are admitted alone).
// * shai_build_decode / shai_build_prefill: per-step device metadata
//   (positions, cache slot mapping, padded block tables, lengths) built in one
//   pass over flattened per-sequence block lists, so the Python engine does no
//   per-token work.
//
// Plays the role of vLLM's scheduler inside the reference's `LLM` engine
// (app/vllm_model_api.py:127-129, is_continuous_batching in
// cova/mllama-32-11b-vllm-trn1-config.yaml:18).
#include <algorithm>
#include <cstdint>

static constexpr int kBlock = 64;

extern "C" {

int shai_sched_admit(int n_waiting, const int* prompt_tokens, int free_blocks, int running, int max_seqs,
                     int token_budget, int watermark_blocks) {
  int admitted = 0, tokens = 0, blocks = 0;
  for (int i = 0; i < n_waiting; ++i) {
    if (running + admitted >= max_seqs) break;
    const int need = (prompt_tokens[i] + kBlock) / kBlock;  // prompt + room for the first generated token
    if (blocks + need > free_blocks - watermark_blocks) break;
    if (admitted > 0 && tokens + prompt_tokens[i] > token_budget) break;
    tokens += prompt_tokens[i];
    blocks += need;
    ++admitted;
  }
  return admitted;
}

void shai_build_decode(int B, const int* ctx_before, const int* tables_flat, const int* table_offs, int max_blocks,
                       int* positions, int* slots, int* ctx_lens, int* bt_out) {
  for (int b = 0; b < B; ++b) {
    const int* tb = tables_flat + table_offs[b];
    const int nb = table_offs[b + 1] - table_offs[b];
    const int pos = ctx_before[b];
    positions[b] = pos;
    slots[b] = tb[pos / kBlock] * kBlock + pos % kBlock;
    ctx_lens[b] = pos + 1;
    int* row = bt_out + (int64_t)b * max_blocks;
    const int n = std::min(nb, max_blocks);
    std::copy(tb, tb + n, row);
    std::fill(row + n, row + max_blocks, 0);
  }
}

void shai_build_prefill(int B, int S, const int* n_cached, const int* n_new, const int* tables_flat,
                        const int* table_offs, int max_blocks, int* positions, int* slots, int* ctx_lens,
                        int* q_lens, int* bt_out, int* last_index) {
  for (int b = 0; b < B; ++b) {
    const int* tb = tables_flat + table_offs[b];
    const int nb = table_offs[b + 1] - table_offs[b];
    for (int s = 0; s < S; ++s) {
      const int t = b * S + s;
      if (s < n_new[b]) {
        const int pos = n_cached[b] + s;
        positions[t] = pos;
        slots[t] = tb[pos / kBlock] * kBlock + pos % kBlock;
      } else {
        positions[t] = 0;
        slots[t] = -1;
      }
    }
    ctx_lens[b] = n_cached[b] + n_new[b];
    q_lens[b] = n_new[b];
    last_index[b] = b * S + n_new[b] - 1;
    int* row = bt_out + (int64_t)b * max_blocks;
    const int n = std::min(nb, max_blocks);
    std::copy(tb, tb + n, row);
    std::fill(row + n, row + max_blocks, 0);
  }
}

// Packed (varlen) prefill: the step's T = sum(n_new) tokens are laid out back to back, no padding rows.
// Sequence b owns rows q_start[b] .. q_start[b] + n_new[b] - 1; a decode row is simply a sequence with
// n_new = 1 (its last token, n_cached = length - 1), so prefill chunks and decode rows share one step.
void shai_build_prefill_packed(int B, const int* n_cached, const int* n_new, const int* tables_flat,
                               const int* table_offs, int max_blocks, int* positions, int* slots, int* ctx_lens,
                               int* q_lens, int* q_start, int* bt_out, int* last_index) {
  int t = 0;
  for (int b = 0; b < B; ++b) {
    const int* tb = tables_flat + table_offs[b];
    const int nb = table_offs[b + 1] - table_offs[b];
    q_start[b] = t;
    for (int s = 0; s < n_new[b]; ++s, ++t) {
      const int pos = n_cached[b] + s;
      positions[t] = pos;
      slots[t] = pos / kBlock < nb ? tb[pos / kBlock] * kBlock + pos % kBlock : -1;
    }
    ctx_lens[b] = n_cached[b] + n_new[b];
    q_lens[b] = n_new[b];
    last_index[b] = t - 1;
    int* row = bt_out + (int64_t)b * max_blocks;
    const int n = std::min(nb, max_blocks);
    std::copy(tb, tb + n, row);
    std::fill(row + n, row + max_blocks, 0);
  }
}

}  // extern "C"
