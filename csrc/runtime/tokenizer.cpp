// Native tokenizers: byte-level BPE for the Qwen2-family
// decoder (with an offline trainer, since no vocabulary files can be
// downloaded) and BERT WordPiece for the encoders (with a hashing fallback
// when no vocab.txt is present).  When real tokenizer files exist the Python
// layer loads them instead; these keep the whole pipeline runnable offline.
#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

enum CharClass { kSpace, kLetter, kDigit, kOther };

inline CharClass cls(unsigned char c) {
  if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v') return kSpace;
  if (std::isalpha(c) || c >= 0x80 || c == '_') return kLetter;
  if (std::isdigit(c)) return kDigit;
  return kOther;
}

// GPT-2 style pre-tokenisation (ASCII approximation): " ?letters", " ?digits",
// " ?punct+", newline runs, and whitespace runs not followed by a word.
void pretokenize(const char* s, size_t n, std::vector<std::pair<size_t, size_t>>& out) {
  size_t i = 0;
  while (i < n) {
    const size_t st = i;
    unsigned char c = (unsigned char)s[i];
    if (c == ' ' && i + 1 < n && cls((unsigned char)s[i + 1]) != kSpace) {
      ++i;
      c = (unsigned char)s[i];
    }
    const CharClass k = cls(c);
    if (k == kSpace) {
      size_t j = i;
      while (j < n && cls((unsigned char)s[j]) == kSpace) ++j;
      // leave one space to attach to the following word
      if (j < n && j - i > 1 && s[j - 1] == ' ') --j;
      i = j;
    } else if (k == kDigit) {
      size_t j = i, cnt = 0;
      while (j < n && cls((unsigned char)s[j]) == kDigit && cnt < 3) ++j, ++cnt;
      i = j;
    } else {
      size_t j = i;
      while (j < n && cls((unsigned char)s[j]) == k) ++j;
      i = j;
    }
    if (i == st) ++i;
    out.emplace_back(st, i - st);
  }
}

struct BPE {
  std::vector<std::pair<int, int>> merges;
  std::unordered_map<uint64_t, int> rank;  // (a<<32|b) -> merge rank
  std::vector<std::string> specials;
  std::vector<int> special_ids;
  std::vector<std::string> vocab;  // id -> bytes

  static uint64_t key(int a, int b) { return ((uint64_t)(uint32_t)a << 32) | (uint32_t)b; }

  void rebuild() {
    vocab.clear();
    for (int i = 0; i < 256; ++i) vocab.push_back(std::string(1, (char)i));
    rank.clear();
    for (size_t r = 0; r < merges.size(); ++r) {
      rank[key(merges[r].first, merges[r].second)] = (int)r;
      vocab.push_back(vocab[merges[r].first] + vocab[merges[r].second]);
    }
  }

  void encode_word(const unsigned char* p, size_t n, std::vector<int>& out) const {
    std::vector<int> w(p, p + n);
    while (w.size() > 1) {
      int best = -1;
      size_t bi = 0;
      for (size_t i = 0; i + 1 < w.size(); ++i) {
        auto it = rank.find(key(w[i], w[i + 1]));
        if (it != rank.end() && (best < 0 || it->second < best)) {
          best = it->second;
          bi = i;
        }
      }
      if (best < 0) break;
      const int a = merges[best].first, b = merges[best].second, nid = 256 + best;
      std::vector<int> nw;
      nw.reserve(w.size());
      for (size_t i = 0; i < w.size();) {
        if (i + 1 < w.size() && w[i] == a && w[i + 1] == b) {
          nw.push_back(nid);
          i += 2;
        } else {
          nw.push_back(w[i]);
          i += 1;
        }
      }
      (void)bi;
      w.swap(nw);
    }
    out.insert(out.end(), w.begin(), w.end());
  }

  void encode(const char* s, size_t n, std::vector<int>& out) const {
    size_t i = 0;
    while (i < n) {
      // earliest special token occurrence
      size_t best_pos = n, best_len = 0;
      int best_id = -1;
      for (size_t k = 0; k < specials.size(); ++k) {
        const std::string& sp = specials[k];
        const char* f = std::search(s + i, s + n, sp.begin(), sp.end());
        const size_t pos = (size_t)(f - s);
        if (pos < best_pos) {
          best_pos = pos;
          best_len = sp.size();
          best_id = special_ids[k];
        }
      }
      const size_t end = best_pos;
      std::vector<std::pair<size_t, size_t>> pieces;
      pretokenize(s + i, end - i, pieces);
      for (auto& pc : pieces) encode_word((const unsigned char*)s + i + pc.first, pc.second, out);
      if (best_id >= 0) {
        out.push_back(best_id);
        i = best_pos + best_len;
      } else {
        i = n;
      }
    }
  }
};

// Greedy BPE training over pre-tokenised word counts.
void train_bpe(BPE& bpe, const char* text, size_t n, int num_merges) {
  std::vector<std::pair<size_t, size_t>> pieces;
  pretokenize(text, n, pieces);
  std::unordered_map<std::string, int> wc;
  for (auto& pc : pieces) wc[std::string(text + pc.first, pc.second)]++;
  std::vector<std::vector<int>> words;
  std::vector<int> counts;
  for (auto& kv : wc) {
    words.emplace_back(kv.first.begin(), kv.first.end());
    for (auto& x : words.back()) x &= 0xFF;
    counts.push_back(kv.second);
  }
  bpe.merges.clear();
  for (int m = 0; m < num_merges; ++m) {
    std::unordered_map<uint64_t, int64_t> pc;
    for (size_t w = 0; w < words.size(); ++w)
      for (size_t i = 0; i + 1 < words[w].size(); ++i) pc[BPE::key(words[w][i], words[w][i + 1])] += counts[w];
    uint64_t best = 0;
    int64_t bc = 1;
    for (auto& kv : pc)
      if (kv.second > bc || (kv.second == bc && kv.first < best)) {
        bc = kv.second;
        best = kv.first;
      }
    if (bc < 2) break;
    const int a = (int)(best >> 32), b = (int)(best & 0xFFFFFFFFu), nid = 256 + m;
    bpe.merges.emplace_back(a, b);
    for (auto& w : words) {
      std::vector<int> nw;
      nw.reserve(w.size());
      for (size_t i = 0; i < w.size();) {
        if (i + 1 < w.size() && w[i] == a && w[i + 1] == b) {
          nw.push_back(nid);
          i += 2;
        } else {
          nw.push_back(w[i++]);
        }
      }
      w.swap(nw);
    }
  }
  bpe.rebuild();
}

// ---------------- WordPiece ----------------
struct WordPiece {
  std::unordered_map<std::string, int> vocab;
  int unk = 100, vocab_size = 30522, hash_offset = 1000;
  bool hashing = true;
  bool lowercase = true;

  static uint64_t fnv(const std::string& s) {
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
    return h;
  }

  void basic(const char* s, size_t n, std::vector<std::string>& toks) const {
    std::string cur;
    auto flush = [&]() {
      if (!cur.empty()) toks.push_back(cur), cur.clear();
    };
    for (size_t i = 0; i < n; ++i) {
      unsigned char c = (unsigned char)s[i];
      if (cls(c) == kSpace) {
        flush();
      } else if (cls(c) == kOther) {
        flush();
        toks.push_back(std::string(1, (char)c));
      } else {
        cur.push_back(lowercase ? (char)std::tolower(c) : (char)c);
      }
    }
    flush();
  }

  void encode(const char* s, size_t n, std::vector<int>& out) const {
    std::vector<std::string> toks;
    basic(s, n, toks);
    for (auto& t : toks) {
      if (hashing) {
        out.push_back(hash_offset + (int)(fnv(t) % (uint64_t)(vocab_size - hash_offset)));
        continue;
      }
      if (t.size() > 100) {
        out.push_back(unk);
        continue;
      }
      std::vector<int> sub;
      size_t st = 0;
      bool bad = false;
      while (st < t.size()) {
        size_t en = t.size();
        int cur = -1;
        while (st < en) {
          std::string piece = t.substr(st, en - st);
          if (st > 0) piece = "##" + piece;
          auto it = vocab.find(piece);
          if (it != vocab.end()) {
            cur = it->second;
            break;
          }
          --en;
        }
        if (cur < 0) {
          bad = true;
          break;
        }
        sub.push_back(cur);
        st = en;
      }
      if (bad) out.push_back(unk);
      else out.insert(out.end(), sub.begin(), sub.end());
    }
  }
};

}  // namespace

extern "C" {

// ---- BPE ----
void* grag_bpe_create() { auto* b = new BPE(); b->rebuild(); return b; }
void grag_bpe_destroy(void* p) { delete static_cast<BPE*>(p); }
int grag_bpe_train(void* p, const char* text, int64_t n, int num_merges) {
  auto* b = static_cast<BPE*>(p);
  train_bpe(*b, text, (size_t)n, num_merges);
  return (int)b->merges.size();
}
// merges as flat int pairs
void grag_bpe_set_merges(void* p, const int32_t* pairs, int n) {
  auto* b = static_cast<BPE*>(p);
  b->merges.clear();
  for (int i = 0; i < n; ++i) b->merges.emplace_back(pairs[2 * i], pairs[2 * i + 1]);
  b->rebuild();
}
int grag_bpe_get_merges(void* p, int32_t* pairs, int cap) {
  auto* b = static_cast<BPE*>(p);
  const int n = (int)b->merges.size();
  for (int i = 0; i < n && i < cap; ++i) {
    pairs[2 * i] = b->merges[i].first;
    pairs[2 * i + 1] = b->merges[i].second;
  }
  return n;
}
void grag_bpe_add_special(void* p, const char* tok, int id) {
  auto* b = static_cast<BPE*>(p);
  b->specials.emplace_back(tok);
  b->special_ids.push_back(id);
}
int grag_bpe_vocab_size(void* p) { return (int)static_cast<BPE*>(p)->vocab.size(); }
// returns number of ids (may exceed cap: caller retries with a bigger buffer)
int64_t grag_bpe_encode(void* p, const char* text, int64_t n, int32_t* out, int64_t cap) {
  auto* b = static_cast<BPE*>(p);
  std::vector<int> ids;
  b->encode(text, (size_t)n, ids);
  for (size_t i = 0; i < ids.size() && (int64_t)i < cap; ++i) out[i] = ids[i];
  return (int64_t)ids.size();
}
// decode to bytes; ids outside the vocab (e.g. random-init sampling) are skipped
int64_t grag_bpe_decode(void* p, const int32_t* ids, int64_t n, char* out, int64_t cap) {
  auto* b = static_cast<BPE*>(p);
  std::string s;
  for (int64_t i = 0; i < n; ++i) {
    const int id = ids[i];
    if (id >= 0 && id < (int)b->vocab.size()) {
      s += b->vocab[id];
    } else {
      for (size_t k = 0; k < b->special_ids.size(); ++k)
        if (b->special_ids[k] == id) s += b->specials[k];
    }
  }
  const int64_t m = (int64_t)s.size();
  if (cap > 0) std::memcpy(out, s.data(), (size_t)std::min(m, cap));
  return m;
}

// ---- WordPiece ----
void* grag_wp_create(int vocab_size, int unk_id, int lowercase) {
  auto* w = new WordPiece();
  w->vocab_size = vocab_size;
  w->unk = unk_id;
  w->lowercase = lowercase != 0;
  return w;
}
void grag_wp_destroy(void* p) { delete static_cast<WordPiece*>(p); }
// vocab: newline-separated tokens, line number = id
void grag_wp_load_vocab(void* p, const char* buf, int64_t n) {
  auto* w = static_cast<WordPiece*>(p);
  w->vocab.clear();
  int id = 0;
  size_t st = 0;
  for (size_t i = 0; i <= (size_t)n; ++i) {
    if (i == (size_t)n || buf[i] == '\n') {
      std::string t(buf + st, i - st);
      if (!t.empty() && t.back() == '\r') t.pop_back();
      if (i < (size_t)n || !t.empty()) w->vocab[t] = id++;
      st = i + 1;
    }
  }
  w->hashing = w->vocab.empty();
}
int64_t grag_wp_encode(void* p, const char* text, int64_t n, int32_t* out, int64_t cap) {
  auto* w = static_cast<WordPiece*>(p);
  std::vector<int> ids;
  w->encode(text, (size_t)n, ids);
  for (size_t i = 0; i < ids.size() && (int64_t)i < cap; ++i) out[i] = ids[i];
  return (int64_t)ids.size();
}

}  // extern "C"
