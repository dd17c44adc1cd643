// Host-runtime self test, built with -fsanitize=address,undefined and with
// -fsanitize=thread by tests/test_native_sanitizers.py (the
// reference has no race detection or sanitizers at all).
//
//  * byte-level BPE: train, encode/decode round trip of ASCII / multi-byte
//    UTF-8 / arbitrary bytes, short output buffers (the "returns the needed
//    size" contract), ids outside the vocabulary, special tokens;
//  * WordPiece: hashing and loaded-vocab modes, truncation capacity;
//  * paged-KV block allocator: 8 threads allocating / freeing / sharing
//    prefixes (match + register) concurrently, then every block accounted for;
//  * concurrent encodes on one shared BPE (the engine thread and the job
//    threads tokenize at the same time; encode is const).
// Exit status 0 = all checks passed (sanitizer reports also fail the test).
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* grag_bpe_create();
void grag_bpe_destroy(void*);
int grag_bpe_train(void*, const char*, int64_t, int);
void grag_bpe_add_special(void*, const char*, int);
int grag_bpe_vocab_size(void*);
int64_t grag_bpe_encode(void*, const char*, int64_t, int32_t*, int64_t);
int64_t grag_bpe_decode(void*, const int32_t*, int64_t, char*, int64_t);
void* grag_wp_create(int, int, int);
void grag_wp_destroy(void*);
void grag_wp_load_vocab(void*, const char*, int64_t);
int64_t grag_wp_encode(void*, const char*, int64_t, int32_t*, int64_t);
void* grag_alloc_create(int, int);
void grag_alloc_destroy(void*);
int grag_alloc_num_free(void*);
int grag_alloc_allocate(void*, int, int32_t*);
void grag_alloc_free(void*, int, const int32_t*);
uint64_t grag_hash_block(uint64_t, const int32_t*, int);
int grag_alloc_match_prefix(void*, const int32_t*, int, int32_t*, uint64_t*);
void grag_alloc_register(void*, int, uint64_t);
int grag_alloc_refcount(void*, int);
}

static int g_fail = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                         \
    }                                                                   \
  } while (0)

static std::string roundtrip(void* bpe, const std::string& s) {
  std::vector<int32_t> ids(4);
  int64_t n = grag_bpe_encode(bpe, s.data(), (int64_t)s.size(), ids.data(), (int64_t)ids.size());
  if (n > (int64_t)ids.size()) {  // short buffer: retry with the size it asked for
    ids.resize((size_t)n);
    CHECK(grag_bpe_encode(bpe, s.data(), (int64_t)s.size(), ids.data(), n) == n);
  }
  ids.resize((size_t)n);
  std::vector<char> buf(3);
  int64_t m = grag_bpe_decode(bpe, ids.data(), n, buf.data(), (int64_t)buf.size());
  if (m > (int64_t)buf.size()) {
    buf.resize((size_t)m);
    CHECK(grag_bpe_decode(bpe, ids.data(), n, buf.data(), m) == m);
  }
  return std::string(buf.data(), (size_t)m);
}

static void test_bpe() {
  void* bpe = grag_bpe_create();
  std::string corpus;
  for (int i = 0; i < 50; ++i)
    corpus += "def retry(policy, timeout=30):\n    return backoff(policy) # exponential backoff\n"
              "The cache is invalidated when the user logs out. ";
  CHECK(grag_bpe_train(bpe, corpus.data(), (int64_t)corpus.size(), 300) > 0);
  grag_bpe_add_special(bpe, "<|im_start|>", 100000);
  grag_bpe_add_special(bpe, "<|im_end|>", 100001);
  const char* cases[] = {"", "a", "def retry(policy):", "naïve café – 日本語 🚀", "\xff\xfe\x00\x01 raw", "  \n\t "};
  for (const char* c : cases) {
    std::string s = std::strcmp(c, "\xff\xfe\x00\x01 raw") == 0 ? std::string(c, 9) : std::string(c);
    CHECK(roundtrip(bpe, s) == s);
  }
  std::mt19937 rng(7);
  for (int t = 0; t < 200; ++t) {  // random byte strings
    std::string s(rng() % 300, '\0');
    for (auto& ch : s) ch = (char)(rng() & 0xff);
    CHECK(roundtrip(bpe, s) == s);
  }
  // specials are matched as single tokens and decode back
  std::string sp = "<|im_start|>user\nhi<|im_end|>";
  CHECK(roundtrip(bpe, sp) == sp);
  // ids outside the vocab are skipped, never read out of bounds
  int32_t bad[4] = {-5, 1 << 30, 65, grag_bpe_vocab_size(bpe)};
  char out[16];
  CHECK(grag_bpe_decode(bpe, bad, 4, out, sizeof(out)) == 1 && out[0] == 'A');
  grag_bpe_destroy(bpe);
}

static void test_wordpiece() {
  void* wp = grag_wp_create(30522, 100, 1);
  int32_t ids[8];
  const std::string s = "Hello World, retry policies with exponential backoff!";
  int64_t n = grag_wp_encode(wp, s.data(), (int64_t)s.size(), ids, 8);
  CHECK(n >= 8);  // full length reported even when truncated to the buffer
  for (int i = 0; i < 8; ++i) CHECK(ids[i] >= 0 && ids[i] < 30522);
  const std::string vocab = "[PAD]\n[UNK]\nhello\nworld\n##s\nretry\n";
  grag_wp_load_vocab(wp, vocab.data(), (int64_t)vocab.size());
  std::vector<int32_t> v(64);
  n = grag_wp_encode(wp, s.data(), (int64_t)s.size(), v.data(), 64);
  CHECK(n > 0 && n <= 64);
  grag_wp_destroy(wp);
}

static void test_allocator_concurrent() {
  const int NB = 4096, BS = 16, T = 8;
  void* al = grag_alloc_create(NB, BS);
  CHECK(grag_alloc_num_free(al) == NB);
  std::atomic<int> errors{0};
  auto worker = [&](int tid) {
    std::mt19937 rng(tid * 977 + 1);
    std::vector<int32_t> toks(BS * 8);
    for (int it = 0; it < 3000; ++it) {
      // a prompt: shared system prefix (4 blocks) + a per-thread tail
      for (int i = 0; i < (int)toks.size(); ++i) toks[i] = i < 4 * BS ? i : (int32_t)(rng() % 50000);
      int32_t got[8];
      uint64_t hs[8];
      const int m = grag_alloc_match_prefix(al, toks.data(), (int)toks.size(), got, hs);
      if (m < 0 || m > 8) errors++;
      int32_t fresh[8];
      const int want = 8 - m;
      if (grag_alloc_allocate(al, want, fresh) != 0) {  // pool exhausted: release the matches
        grag_alloc_free(al, m, got);
        continue;
      }
      uint64_t parent = m ? hs[m - 1] : 0;
      for (int j = 0; j < want; ++j) {
        const int blk = m + j;
        parent = grag_hash_block(parent, toks.data() + blk * BS, BS);
        if (rng() & 1) grag_alloc_register(al, fresh[j], parent);
      }
      for (int j = 0; j < m; ++j)
        if (grag_alloc_refcount(al, got[j]) < 1) errors++;
      grag_alloc_free(al, m, got);
      grag_alloc_free(al, want, fresh);
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back(worker, t);
  for (auto& x : th) x.join();
  CHECK(errors.load() == 0);
  // everything returned: free plain + evictable cached blocks cover the pool
  CHECK(grag_alloc_num_free(al) == NB);
  for (int b = 0; b < NB; ++b) CHECK(grag_alloc_refcount(al, b) == 0);
  int32_t all[NB];
  CHECK(grag_alloc_allocate(al, NB, all) == 0);  // cached blocks are evicted on demand
  CHECK(grag_alloc_allocate(al, 1, all) == -1);
  grag_alloc_free(al, NB, all);
  grag_alloc_destroy(al);
}

static void test_concurrent_encode() {
  void* bpe = grag_bpe_create();
  std::string corpus(20000, 'x');
  for (size_t i = 0; i < corpus.size(); ++i) corpus[i] = "abcdefgh ij\n"[i % 12];
  grag_bpe_train(bpe, corpus.data(), (int64_t)corpus.size(), 200);
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      std::string s = "thread " + std::to_string(t) + " abcdefgh ij abcdefgh";
      for (int i = 0; i < 500; ++i)
        if (roundtrip(bpe, s) != s) bad++;
    });
  for (auto& x : th) x.join();
  CHECK(bad.load() == 0);
  grag_bpe_destroy(bpe);
}

int main() {
  test_bpe();
  test_wordpiece();
  test_allocator_concurrent();
  test_concurrent_encode();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("runtime selftest ok\n");
  return 0;
}
