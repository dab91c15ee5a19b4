// Host sanitizer driver for the native runtime (race detection / sanitizers).
//
// Built by tests/test_runtime_sanitizers_cpu.py three ways -- plain, -fsanitize=address,undefined
// and -fsanitize=thread -- and linked directly against block_manager.cpp + scheduler.cpp:
//
// * T threads hammer ONE block manager concurrently (allocate / fork / release / register /
//   prefix lookup) the way the engine thread and API threads can; TSan reports any access to
//   the shared state outside the mutex, ASan/UBSan any out-of-bounds or lifetime bug.
// * After the threads join, the block accounting must balance: every block is free, cached
//   (LRU) or referenced, and all refcounts are back to zero.
// * shai_build_decode / shai_build_prefill are run on random ragged block tables and checked
//   against a direct recomputation of positions / slots / lengths.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

extern "C" {
void* shai_bm_create(int num_blocks);
void shai_bm_destroy(void* h);
int shai_bm_num_free(void* h);
int shai_bm_num_blocks(void* h);
int shai_bm_allocate(void* h, int n, int* out);
void shai_bm_fork(void* h, const int* blocks, int n);
void shai_bm_release(void* h, const int* blocks, int n);
void shai_bm_register(void* h, int block, uint64_t content_hash);
int shai_bm_lookup_prefix(void* h, const uint64_t* hashes, int n, int* out);
void shai_bm_stats(void* h, int64_t* out);
int shai_bm_refcount(void* h, int block);
int shai_sched_admit(int n_waiting, const int* prompt_tokens, int free_blocks, int running, int max_seqs,
                     int token_budget, int watermark_blocks);
void shai_build_decode(int B, const int* ctx_before, const int* tables_flat, const int* table_offs, int max_blocks,
                       int* positions, int* slots, int* ctx_lens, int* bt_out);
void shai_build_prefill(int B, int S, const int* n_cached, const int* n_new, const int* tables_flat,
                        const int* table_offs, int max_blocks, int* positions, int* slots, int* ctx_lens,
                        int* q_lens, int* bt_out, int* last_index);
}

static constexpr int kBlock = 64;
static int g_fail = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                       \
    }                                                                 \
  } while (0)

static void worker(void* bm, int tid, int iters) {
  std::mt19937 rng(1234 + tid);
  std::vector<std::vector<int>> held;
  for (int it = 0; it < iters; ++it) {
    const int op = rng() % 5;
    if (op <= 1) {  // allocate a sequence's worth of blocks, maybe register some as "full" cached blocks
      const int n = 1 + rng() % 6;
      std::vector<int> b(n);
      if (shai_bm_allocate(bm, n, b.data()) == 0) {
        for (int i = 0; i < n; ++i) {
          CHECK(b[i] >= 0 && b[i] < shai_bm_num_blocks(bm));
          if (rng() % 3 == 0) shai_bm_register(bm, b[i], 1 + (uint64_t)(rng() % 97));  // shared hash space
        }
        held.push_back(std::move(b));
      }
    } else if (op == 2 && !held.empty()) {  // fork (shared prefix): one more reference on the same blocks
      auto b = held[rng() % held.size()];
      shai_bm_fork(bm, b.data(), (int)b.size());
      held.push_back(std::move(b));
    } else if (op == 3 && !held.empty()) {  // finish a sequence
      const size_t i = rng() % held.size();
      shai_bm_release(bm, held[i].data(), (int)held[i].size());
      held[i] = std::move(held.back());
      held.pop_back();
    } else {  // prefix-cache lookup; found blocks get a reference we must drop again
      uint64_t hs[4];
      for (auto& h : hs) h = 1 + (uint64_t)(rng() % 97);
      int out[4];
      const int f = shai_bm_lookup_prefix(bm, hs, 4, out);
      CHECK(f >= 0 && f <= 4);
      if (f > 0) held.emplace_back(out, out + f);
    }
    if (it % 64 == 0) {
      int64_t st[4];
      shai_bm_stats(bm, st);
      CHECK(st[0] <= st[1]);
    }
  }
  for (auto& b : held) shai_bm_release(bm, b.data(), (int)b.size());
}

static void check_builders(std::mt19937& rng) {
  for (int trial = 0; trial < 200; ++trial) {
    const int B = 1 + rng() % 9, max_blocks = 1 + rng() % 12;
    std::vector<int> offs(B + 1, 0), flat, ctx(B);
    for (int b = 0; b < B; ++b) {
      const int nb = 1 + rng() % max_blocks;
      for (int i = 0; i < nb; ++i) flat.push_back(rng() % 4096);
      offs[b + 1] = (int)flat.size();
      ctx[b] = rng() % (nb * kBlock);  // next token lands inside the allocated blocks
    }
    std::vector<int> pos(B), slots(B), lens(B), bt((size_t)B * max_blocks, -7);
    shai_build_decode(B, ctx.data(), flat.data(), offs.data(), max_blocks, pos.data(), slots.data(), lens.data(),
                      bt.data());
    for (int b = 0; b < B; ++b) {
      CHECK(pos[b] == ctx[b] && lens[b] == ctx[b] + 1);
      CHECK(slots[b] == flat[offs[b] + ctx[b] / kBlock] * kBlock + ctx[b] % kBlock);
      const int nb = offs[b + 1] - offs[b];
      for (int i = 0; i < max_blocks; ++i) CHECK(bt[(size_t)b * max_blocks + i] == (i < nb ? flat[offs[b] + i] : 0));
    }
    // prefill: S-padded rows of new tokens after n_cached cached ones
    const int S = 1 + rng() % 80;
    std::vector<int> nc(B), nn(B);
    for (int b = 0; b < B; ++b) {
      const int cap = (offs[b + 1] - offs[b]) * kBlock;
      nn[b] = 1 + rng() % std::min(S, cap);
      nc[b] = rng() % (cap - nn[b] + 1);
    }
    std::vector<int> ppos((size_t)B * S), pslots((size_t)B * S), plens(B), qlens(B), last(B),
        pbt((size_t)B * max_blocks);
    shai_build_prefill(B, S, nc.data(), nn.data(), flat.data(), offs.data(), max_blocks, ppos.data(), pslots.data(),
                       plens.data(), qlens.data(), pbt.data(), last.data());
    for (int b = 0; b < B; ++b) {
      CHECK(plens[b] == nc[b] + nn[b] && qlens[b] == nn[b] && last[b] == b * S + nn[b] - 1);
      for (int s = 0; s < S; ++s) {
        const size_t t = (size_t)b * S + s;
        if (s < nn[b]) {
          const int p = nc[b] + s;
          CHECK(ppos[t] == p && pslots[t] == flat[offs[b] + p / kBlock] * kBlock + p % kBlock);
        } else {
          CHECK(pslots[t] == -1);
        }
      }
    }
  }
  // admission budgets
  std::vector<int> prompts = {100, 30, 500, 64, 64};
  CHECK(shai_sched_admit(5, prompts.data(), 1000, 0, 2, 1 << 20, 0) == 2);           // max_seqs
  CHECK(shai_sched_admit(5, prompts.data(), 3, 0, 64, 1 << 20, 0) == 2);             // blocks: 2 + 1 fit, +8 not
  CHECK(shai_sched_admit(5, prompts.data(), 1000, 0, 64, 120, 0) == 1);              // token budget (first always)
  CHECK(shai_sched_admit(0, prompts.data(), 1000, 0, 64, 120, 0) == 0);
}

int main(int argc, char** argv) {
  const int threads = argc > 1 ? std::atoi(argv[1]) : 4;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 20000;
  const int nblocks = 256;
  void* bm = shai_bm_create(nblocks);
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) ts.emplace_back(worker, bm, t, iters);
  for (auto& t : ts) t.join();
  // every reference dropped: all blocks free or parked in the prefix-cache LRU
  CHECK(shai_bm_num_free(bm) == nblocks);
  for (int b = 0; b < nblocks; ++b) CHECK(shai_bm_refcount(bm, b) == 0);
  CHECK(shai_bm_refcount(bm, -1) == -1 && shai_bm_refcount(bm, nblocks) == -1);
  int64_t st[4];
  shai_bm_stats(bm, st);
  CHECK(st[2] + st[3] == nblocks);
  // a full drain must evict every cached block without losing any
  std::vector<int> all(nblocks);
  CHECK(shai_bm_allocate(bm, nblocks, all.data()) == 0);
  CHECK(shai_bm_num_free(bm) == 0);
  int extra;
  CHECK(shai_bm_allocate(bm, 1, &extra) == -1);
  shai_bm_release(bm, all.data(), nblocks);
  CHECK(shai_bm_num_free(bm) == nblocks);
  shai_bm_destroy(bm);

  std::mt19937 rng(7);
  check_builders(rng);
  if (g_fail) {
    std::fprintf(stderr, "%d checks failed\n", g_fail);
    return 1;
  }
  std::printf("runtime stress ok (threads=%d iters=%d)\n", threads, iters);
  return 0;
}
