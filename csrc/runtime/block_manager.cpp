// Paged-KV block manager (host C++, C ABI for ctypes).
//
// Owns the 64-token KV blocks of one engine replica: a free stack, per-block
// reference counts (sequences sharing a prefix / forked sequences share
// blocks), and a hash -> block prefix cache of FULL blocks.  A released block
// whose content is hashed is parked in an LRU "evictable" list instead of the
// free stack, so a later request with the same prompt prefix reuses the
// already-computed K/V (prefix caching); allocation evicts LRU cached blocks
// only when the free stack is empty.
//
// The reference delegates this to vLLM's (Neuron fork) block manager behind
// `LLM(**vllm_config)` (app/vllm_model_api.py:127-129; block_size in
// cova/mllama-32-11b-vllm-trn1-config.yaml:7-23).
#include <cstdint>
#include <list>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

struct BlockManager {
  int num_blocks;
  std::vector<int> free_stack;
  std::vector<int> refcnt;
  std::vector<uint64_t> hash;   // 0 = not a cached full block
  std::vector<char> has_hash;
  std::unordered_map<uint64_t, int> cache;  // content hash -> block
  std::list<int> lru;                       // evictable cached blocks (front = oldest)
  std::vector<std::list<int>::iterator> lru_it;
  std::vector<char> in_lru;
  std::mutex mu;
  int64_t hits = 0, queries = 0;

  explicit BlockManager(int n)
      : num_blocks(n), refcnt(n, 0), hash(n, 0), has_hash(n, 0), lru_it(n), in_lru(n, 0) {
    free_stack.reserve(n);
    for (int i = n - 1; i >= 0; --i) free_stack.push_back(i);
  }

  void drop_hash(int b) {
    if (has_hash[b]) {
      auto it = cache.find(hash[b]);
      if (it != cache.end() && it->second == b) cache.erase(it);
      has_hash[b] = 0;
      hash[b] = 0;
    }
  }

  int take_one() {
    if (!free_stack.empty()) {
      int b = free_stack.back();
      free_stack.pop_back();
      return b;
    }
    if (!lru.empty()) {
      int b = lru.front();
      lru.pop_front();
      in_lru[b] = 0;
      drop_hash(b);
      return b;
    }
    return -1;
  }
};

}  // namespace

extern "C" {

void* shai_bm_create(int num_blocks) { return new BlockManager(num_blocks); }

void shai_bm_destroy(void* h) { delete static_cast<BlockManager*>(h); }

int shai_bm_num_free(void* h) {
  auto* m = static_cast<BlockManager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  return (int)(m->free_stack.size() + m->lru.size());
}

int shai_bm_num_blocks(void* h) { return static_cast<BlockManager*>(h)->num_blocks; }

// Allocate n blocks (refcount 1). Returns 0 on success, -1 (nothing allocated) if short.
int shai_bm_allocate(void* h, int n, int* out) {
  auto* m = static_cast<BlockManager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  if ((int)(m->free_stack.size() + m->lru.size()) < n) return -1;
  for (int i = 0; i < n; ++i) {
    int b = m->take_one();
    m->refcnt[b] = 1;
    out[i] = b;
  }
  return 0;
}

// Increment reference counts (sequence fork / shared prefix).
void shai_bm_fork(void* h, const int* blocks, int n) {
  auto* m = static_cast<BlockManager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  for (int i = 0; i < n; ++i) {
    int b = blocks[i];
    if (b < 0 || b >= m->num_blocks) continue;
    if (m->in_lru[b]) {
      m->lru.erase(m->lru_it[b]);
      m->in_lru[b] = 0;
    }
    m->refcnt[b] += 1;
  }
}

// Decrement; blocks reaching zero go to the LRU (if content-hashed) or the free stack.
void shai_bm_release(void* h, const int* blocks, int n) {
  auto* m = static_cast<BlockManager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  for (int i = n - 1; i >= 0; --i) {
    int b = blocks[i];
    if (b < 0 || b >= m->num_blocks || m->refcnt[b] <= 0) continue;
    if (--m->refcnt[b] == 0) {
      if (m->has_hash[b]) {
        m->lru.push_back(b);
        m->lru_it[b] = std::prev(m->lru.end());
        m->in_lru[b] = 1;
      } else {
        m->free_stack.push_back(b);
      }
    }
  }
}

// Mark a full block's content hash (chained over the prefix by the caller).
void shai_bm_register(void* h, int block, uint64_t content_hash) {
  auto* m = static_cast<BlockManager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  if (block < 0 || block >= m->num_blocks) return;
  if (m->cache.count(content_hash)) return;  // another block already caches it
  m->drop_hash(block);
  m->hash[block] = content_hash;
  m->has_hash[block] = 1;
  m->cache[content_hash] = block;
}

// Longest cached prefix: for i in order, hashes[i] -> block; stops at the first miss.
// Found blocks get a reference. Returns the number of blocks found.
int shai_bm_lookup_prefix(void* h, const uint64_t* hashes, int n, int* out) {
  auto* m = static_cast<BlockManager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  int found = 0;
  m->queries += n;
  for (int i = 0; i < n; ++i) {
    auto it = m->cache.find(hashes[i]);
    if (it == m->cache.end()) break;
    int b = it->second;
    if (m->in_lru[b]) {
      m->lru.erase(m->lru_it[b]);
      m->in_lru[b] = 0;
    }
    m->refcnt[b] += 1;
    out[found++] = b;
  }
  m->hits += found;
  return found;
}

void shai_bm_stats(void* h, int64_t* out) {
  auto* m = static_cast<BlockManager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  out[0] = m->hits;
  out[1] = m->queries;
  out[2] = (int64_t)m->free_stack.size();
  out[3] = (int64_t)m->lru.size();
}

int shai_bm_refcount(void* h, int block) {
  auto* m = static_cast<BlockManager*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  return (block < 0 || block >= m->num_blocks) ? -1 : m->refcnt[block];
}

}  // extern "C"
