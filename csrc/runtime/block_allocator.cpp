// Paged-KV block allocator with content-hash prefix caching (host C++).
//
// Replaces what the reference reached through vLLM's block manager
// ("paged KV block manager (C++)").  Blocks are fixed-size
// token pages of the device KV cache.  A full block whose chained token hash
// is registered can be shared by later sequences with the same prefix (the
// agent's prompts and the ingest extractor waves share long prefixes); freed
// hashed blocks stay cached and are evicted LRU only when the free pool runs
// dry.  Thread-safe (one mutex) so the scheduler thread and API threads can
// query it.
#include <cstdint>
#include <list>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

struct Allocator {
  int num_blocks;
  int block_size;
  std::vector<int> refcnt;
  std::vector<uint64_t> hash_of;  // 0 = unhashed
  std::vector<int> free_plain;    // never-hashed free blocks (LIFO)
  std::list<int> lru;             // hashed blocks with refcnt 0 (front = oldest)
  std::vector<std::list<int>::iterator> lru_pos;
  std::vector<char> in_lru;
  std::unordered_map<uint64_t, int> by_hash;
  std::mutex mu;
  int64_t hits = 0, queries = 0;

  Allocator(int n, int bs)
      : num_blocks(n), block_size(bs), refcnt(n, 0), hash_of(n, 0), lru_pos(n), in_lru(n, 0) {
    free_plain.reserve(n);
    for (int i = n - 1; i >= 0; --i) free_plain.push_back(i);
  }

  int num_free_locked() const { return (int)free_plain.size() + (int)lru.size(); }

  int take_one() {
    if (!free_plain.empty()) {
      const int b = free_plain.back();
      free_plain.pop_back();
      return b;
    }
    if (!lru.empty()) {
      const int b = lru.front();
      lru.pop_front();
      in_lru[b] = 0;
      if (hash_of[b]) {
        auto it = by_hash.find(hash_of[b]);
        if (it != by_hash.end() && it->second == b) by_hash.erase(it);
        hash_of[b] = 0;
      }
      return b;
    }
    return -1;
  }
};

inline uint64_t mix(uint64_t h, uint64_t v) {
  h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
  h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33;
  return h;
}

}  // namespace

extern "C" {

void* grag_alloc_create(int num_blocks, int block_size) { return new Allocator(num_blocks, block_size); }
void grag_alloc_destroy(void* a) { delete static_cast<Allocator*>(a); }

int grag_alloc_num_free(void* a) {
  auto* al = static_cast<Allocator*>(a);
  std::lock_guard<std::mutex> g(al->mu);
  return al->num_free_locked();
}

// Allocate n fresh blocks into out. Returns 0 or -1 (nothing allocated).
int grag_alloc_allocate(void* a, int n, int32_t* out) {
  auto* al = static_cast<Allocator*>(a);
  std::lock_guard<std::mutex> g(al->mu);
  if (n > al->num_free_locked()) return -1;
  for (int i = 0; i < n; ++i) {
    const int b = al->take_one();
    al->refcnt[b] = 1;
    out[i] = b;
  }
  return 0;
}

void grag_alloc_free(void* a, int n, const int32_t* ids) {
  auto* al = static_cast<Allocator*>(a);
  std::lock_guard<std::mutex> g(al->mu);
  for (int i = 0; i < n; ++i) {
    const int b = ids[i];
    if (b < 0 || b >= al->num_blocks || al->refcnt[b] <= 0) continue;
    if (--al->refcnt[b] == 0) {
      if (al->hash_of[b]) {
        al->lru.push_back(b);
        al->lru_pos[b] = std::prev(al->lru.end());
        al->in_lru[b] = 1;
      } else {
        al->free_plain.push_back(b);
      }
    }
  }
}

// Chained hash of one full block of tokens.
uint64_t grag_hash_block(uint64_t parent, const int32_t* toks, int n) {
  uint64_t h = mix(0x243F6A8885A308D3ull, parent);
  for (int i = 0; i < n; ++i) h = mix(h, (uint64_t)(uint32_t)toks[i]);
  return h ? h : 1;
}

// Chained hashes of `nblocks` consecutive full blocks of `bs` tokens (one call for a prompt's blocks).
void grag_hash_blocks(uint64_t parent, const int32_t* toks, int nblocks, int bs, uint64_t* out) {
  for (int b = 0; b < nblocks; ++b) {
    parent = grag_hash_block(parent, toks + (size_t)b * bs, bs);
    out[b] = parent;
  }
}

// grag_alloc_register for n (block, hash) pairs under one lock.
void grag_alloc_register_many(void* a, const int32_t* blocks, const uint64_t* hashes, int n) {
  auto* al = static_cast<Allocator*>(a);
  std::lock_guard<std::mutex> g(al->mu);
  for (int i = 0; i < n; ++i) {
    const int block = blocks[i];
    const uint64_t h = hashes[i];
    if (block < 0 || block >= al->num_blocks || h == 0) continue;
    if (al->by_hash.count(h)) continue;
    if (al->hash_of[block]) continue;
    al->hash_of[block] = h;
    al->by_hash[h] = block;
  }
}

// Drop the hashes of n blocks (a step that registered its prefill blocks at scheduling time failed
// before computing them: the cache must not serve their contents).  Unreferenced ones become plain free.
void grag_alloc_unregister(void* a, int n, const int32_t* blocks) {
  auto* al = static_cast<Allocator*>(a);
  std::lock_guard<std::mutex> g(al->mu);
  for (int i = 0; i < n; ++i) {
    const int b = blocks[i];
    if (b < 0 || b >= al->num_blocks || !al->hash_of[b]) continue;
    auto it = al->by_hash.find(al->hash_of[b]);
    if (it != al->by_hash.end() && it->second == b) al->by_hash.erase(it);
    al->hash_of[b] = 0;
    if (al->in_lru[b]) {
      al->lru.erase(al->lru_pos[b]);
      al->in_lru[b] = 0;
      al->free_plain.push_back(b);
    }
  }
}

// Look up the longest cached prefix of `ntok` tokens. Fills out[] with the
// reused block ids (refcount taken) and returns how many full blocks matched.
int grag_alloc_match_prefix(void* a, const int32_t* toks, int ntok, int32_t* out, uint64_t* hashes_out) {
  auto* al = static_cast<Allocator*>(a);
  std::lock_guard<std::mutex> g(al->mu);
  const int bs = al->block_size;
  uint64_t parent = 0;
  int matched = 0;
  for (int s = 0; s + bs <= ntok; s += bs) {
    const uint64_t h = grag_hash_block(parent, toks + s, bs);
    al->queries++;
    auto it = al->by_hash.find(h);
    if (it == al->by_hash.end()) break;
    const int b = it->second;
    if (al->refcnt[b] == 0 && al->in_lru[b]) {
      al->lru.erase(al->lru_pos[b]);
      al->in_lru[b] = 0;
    }
    al->refcnt[b]++;
    out[matched] = b;
    if (hashes_out) hashes_out[matched] = h;
    matched++;
    al->hits++;
    parent = h;
  }
  return matched;
}

// Register a now-full block under its chained hash (first writer wins).
void grag_alloc_register(void* a, int block, uint64_t h) {
  auto* al = static_cast<Allocator*>(a);
  std::lock_guard<std::mutex> g(al->mu);
  if (block < 0 || block >= al->num_blocks || h == 0) return;
  if (al->by_hash.count(h)) return;
  if (al->hash_of[block]) return;
  al->hash_of[block] = h;
  al->by_hash[h] = block;
}

void grag_alloc_stats(void* a, int64_t* out3) {
  auto* al = static_cast<Allocator*>(a);
  std::lock_guard<std::mutex> g(al->mu);
  out3[0] = al->hits;
  out3[1] = al->queries;
  out3[2] = (int64_t)al->by_hash.size();
}

int grag_alloc_refcount(void* a, int block) {
  auto* al = static_cast<Allocator*>(a);
  std::lock_guard<std::mutex> g(al->mu);
  return (block >= 0 && block < al->num_blocks) ? al->refcnt[block] : -1;
}

}  // extern "C"
