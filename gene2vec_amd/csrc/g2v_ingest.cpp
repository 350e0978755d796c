// g2v_ingest.cpp -- native corpus ingest for libg2v.so (host only).
//
// Replaces the Python ingest of src/gene2vec.py:36-47 and :52/:80:
//   for fname in files: for line in open(f, encoding='windows-1252'):
//       gene_pairs.append(line.strip().split())
//   random.shuffle(gene_pairs)
// with a multi-threaded reader that yields CSR token ids (ids in global
// first-occurrence order over the given file order) and a permutation that
// is bit-identical to CPython's random.Random.shuffle for the same state.
//
// Semantics reproduced exactly:
//  * text mode universal newlines: "\n", "\r\n" and a lone "\r" end a line;
//  * str.split() separators after windows-1252 decoding: the ASCII
//    whitespace " \t\n\v\f\r", the separators 0x1c-0x1f and 0xa0 (U+00A0);
//  * bytes 0x81 0x8d 0x8f 0x90 0x9d are undefined in windows-1252: Python's
//    decoder raises UnicodeDecodeError -> G2V_EINVAL here;
//  * an empty / whitespace-only line is an empty sentence (kept).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <new>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "g2v.h"

namespace {

inline bool is_sep(unsigned char c) {
  return c == ' ' || (c >= 0x09 && c <= 0x0d) || (c >= 0x1c && c <= 0x1f) || c == 0xa0;
}
inline bool is_undefined_cp1252(unsigned char c) {
  return c == 0x81 || c == 0x8d || c == 0x8f || c == 0x90 || c == 0x9d;
}

struct Chunk {  // one file (or a line-aligned piece of one)
  const char* p = nullptr;
  size_t n = 0;
  std::vector<int32_t> tok;              // local ids
  std::vector<int64_t> len;              // sentence lengths
  std::vector<std::string_view> words;   // local id -> bytes (views into the file buffer)
  std::vector<int64_t> cnt;              // local counts
  int err = 0;
  size_t err_at = 0;
};

void tokenize(Chunk& c) {
  std::unordered_map<std::string_view, int32_t> ids;
  ids.reserve(1 << 16);
  const unsigned char* s = (const unsigned char*)c.p;
  size_t i = 0, n = c.n;
  while (i < n) {
    // one line: up to '\n', '\r\n' or '\r'
    int64_t ntok = 0;
    while (i < n && s[i] != '\n' && s[i] != '\r') {
      if (is_sep(s[i])) {
        ++i;
        continue;
      }
      const size_t b = i;
      while (i < n && s[i] != '\n' && s[i] != '\r' && !is_sep(s[i])) {
        if (is_undefined_cp1252(s[i]) && !c.err) {
          c.err = 1;
          c.err_at = i;
        }
        ++i;
      }
      std::string_view w((const char*)s + b, i - b);
      auto it = ids.find(w);
      int32_t id;
      if (it == ids.end()) {
        id = (int32_t)c.words.size();
        ids.emplace(w, id);
        c.words.push_back(w);
        c.cnt.push_back(0);
      } else {
        id = it->second;
      }
      c.cnt[id]++;
      c.tok.push_back(id);
      ++ntok;
    }
    c.len.push_back(ntok);
    if (i < n) {  // consume the line terminator
      if (s[i] == '\r' && i + 1 < n && s[i + 1] == '\n') i += 2;
      else ++i;
    }
  }
}

}  // namespace

struct g2v_corpus {
  std::vector<std::string> files;     // file contents (owned buffers)
  std::vector<int32_t> tok;
  std::vector<int64_t> off;
  std::vector<std::string> words;     // global id -> bytes (windows-1252)
  std::vector<int64_t> counts;
};

extern "C" {

int g2v_corpus_read(const char* const* paths, int n_paths, int n_threads, g2v_corpus** out) {
  if (!out || (n_paths > 0 && !paths) || n_paths < 0) return G2V_EINVAL;
  *out = nullptr;
  g2v_corpus* cp = new (std::nothrow) g2v_corpus();
  if (!cp) return G2V_ENOMEM;
  cp->files.resize(n_paths);
  for (int f = 0; f < n_paths; ++f) {
    FILE* fp = fopen(paths[f], "rb");
    if (!fp) {
      delete cp;
      return G2V_EINVAL;
    }
    fseek(fp, 0, SEEK_END);
    const long sz = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    cp->files[f].resize(sz > 0 ? (size_t)sz : 0);
    if (sz > 0 && fread(&cp->files[f][0], 1, (size_t)sz, fp) != (size_t)sz) {
      fclose(fp);
      delete cp;
      return G2V_EINVAL;
    }
    fclose(fp);
  }
  // line-aligned chunks of ~64 MiB, in file order
  std::vector<Chunk> chunks;
  const size_t target = (size_t)64 << 20;
  for (auto& buf : cp->files) {
    size_t b = 0;
    if (buf.empty()) continue;
    while (b < buf.size()) {
      size_t e = std::min(buf.size(), b + target);
      while (e < buf.size() && buf[e - 1] != '\n' && buf[e - 1] != '\r') ++e;
      // never split a "\r\n" pair
      if (e < buf.size() && buf[e - 1] == '\r' && buf[e] == '\n') ++e;
      Chunk c;
      c.p = buf.data() + b;
      c.n = e - b;
      chunks.push_back(std::move(c));
      b = e;
    }
  }
  const int nt = std::max(1, std::min<int>(n_threads > 0 ? n_threads : 8, (int)chunks.size()));
  {
    std::vector<std::thread> th;
    std::atomic_size_t next{0};
    for (int t = 0; t < nt; ++t)
      th.emplace_back([&]() {
        for (size_t k; (k = next.fetch_add(1)) < chunks.size();) tokenize(chunks[k]);
      });
    for (auto& t : th) t.join();
  }
  for (auto& c : chunks)
    if (c.err) {
      delete cp;
      return G2V_EINVAL;  // UnicodeDecodeError in the reference
    }
  // merge in chunk order: global first occurrence = chunk order + local order
  std::unordered_map<std::string_view, int32_t> gid;
  size_t ntok = 0, nsent = 0;
  for (auto& c : chunks) {
    ntok += c.tok.size();
    nsent += c.len.size();
  }
  cp->tok.resize(ntok);
  cp->off.resize(nsent + 1);
  std::vector<std::string_view> gwords;
  size_t tpos = 0, spos = 0;
  cp->off[0] = 0;
  for (auto& c : chunks) {
    std::vector<int32_t> remap(c.words.size());
    for (size_t l = 0; l < c.words.size(); ++l) {
      auto it = gid.find(c.words[l]);
      if (it == gid.end()) {
        const int32_t g = (int32_t)gwords.size();
        gid.emplace(c.words[l], g);
        gwords.push_back(c.words[l]);
        cp->counts.push_back(0);
        remap[l] = g;
      } else {
        remap[l] = it->second;
      }
      cp->counts[remap[l]] += c.cnt[l];
    }
    for (int32_t t : c.tok) cp->tok[tpos++] = remap[t];
    for (int64_t L : c.len) {
      cp->off[spos + 1] = cp->off[spos] + L;
      ++spos;
    }
  }
  cp->words.reserve(gwords.size());
  for (auto& w : gwords) cp->words.emplace_back(w);
  *out = cp;
  return G2V_OK;
}

int g2v_corpus_info(const g2v_corpus* c, int64_t* n_tokens, int64_t* n_sent, int64_t* n_words,
                    int64_t* word_bytes) {
  if (!c) return G2V_EINVAL;
  if (n_tokens) *n_tokens = (int64_t)c->tok.size();
  if (n_sent) *n_sent = (int64_t)c->off.size() - 1;
  if (n_words) *n_words = (int64_t)c->words.size();
  if (word_bytes) {
    int64_t b = 0;
    for (auto& w : c->words) b += (int64_t)w.size();
    *word_bytes = b;
  }
  return G2V_OK;
}

// tokens[n_tokens], sent_off[n_sent+1], counts[n_words], words as concatenated
// bytes + word_off[n_words+1]; any pointer may be NULL
int g2v_corpus_export(const g2v_corpus* c, int32_t* tokens, int64_t* sent_off, int64_t* counts,
                      char* words, int64_t* word_off) {
  if (!c) return G2V_EINVAL;
  if (tokens) memcpy(tokens, c->tok.data(), c->tok.size() * sizeof(int32_t));
  if (sent_off) memcpy(sent_off, c->off.data(), c->off.size() * sizeof(int64_t));
  if (counts) memcpy(counts, c->counts.data(), c->counts.size() * sizeof(int64_t));
  if (words || word_off) {
    int64_t b = 0;
    for (size_t i = 0; i < c->words.size(); ++i) {
      if (word_off) word_off[i] = b;
      if (words) memcpy(words + b, c->words[i].data(), c->words[i].size());
      b += (int64_t)c->words[i].size();
    }
    if (word_off) word_off[c->words.size()] = b;
  }
  return G2V_OK;
}

int g2v_csr_permute(const int32_t* tok, const int64_t* off, int64_t n_sent, const int64_t* perm,
                    int32_t* out_tok, int64_t* out_off) {
  if (n_sent < 0 || (n_sent > 0 && (!tok || !off || !perm || !out_tok || !out_off)))
    return G2V_EINVAL;
  out_off[0] = 0;
  // lengths (parallel) -> offsets (block-parallel scan) -> gather (parallel)
  const int nt = (int)std::min<int64_t>(16, std::max<int64_t>(1, n_sent >> 16));
  std::atomic<bool> bad{false};
  std::vector<int64_t> part((size_t)nt + 1, 0);
  auto run = [&](auto&& fn) {
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(fn, t);
    fn(0);
    for (auto& x : th) x.join();
  };
  run([&](int t) {
    const int64_t a = n_sent * t / nt, b = n_sent * (t + 1) / nt;
    int64_t sum = 0;
    for (int64_t i = a; i < b; ++i) {
      const int64_t p = perm[i];
      if (p < 0 || p >= n_sent) {
        bad = true;
        return;
      }
      sum += off[p + 1] - off[p];
      out_off[i + 1] = sum;
    }
    part[(size_t)t + 1] = sum;
  });
  if (bad) return G2V_EINVAL;
  for (int t = 0; t < nt; ++t) part[(size_t)t + 1] += part[(size_t)t];
  run([&](int t) {
    const int64_t a = n_sent * t / nt, b = n_sent * (t + 1) / nt;
    const int64_t base = part[(size_t)t];
    for (int64_t i = a; i < b; ++i) {
      out_off[i + 1] += base;
      const int64_t p = perm[i];
      const int64_t len = off[p + 1] - off[p];
      const int32_t* src = tok + off[p];
      int32_t* dst = out_tok + (out_off[i + 1] - len);
      if (len == 2) {
        dst[0] = src[0];
        dst[1] = src[1];
      } else {
        memcpy(dst, src, sizeof(int32_t) * len);
      }
    }
  });
  return G2V_OK;
}

int g2v_corpus_free(g2v_corpus* c) {
  delete c;
  return G2V_OK;
}

// --------------------------------------------------------------------------
// CPython random.Random.shuffle, bit-compatible.  state[0..623] + pos are the
// first 625 ints of random.getstate()[1]; both are updated in place so the
// caller can setstate() afterwards and keep the Python generator in step.
// shuffle(x): for i in reversed(range(1, n)): j = _randbelow(i + 1); swap
// _randbelow(m): k = m.bit_length(); r = getrandbits(k); while r >= m: retry
// getrandbits(k <= 32) = genrand_uint32() >> (32 - k)
// --------------------------------------------------------------------------
namespace {
struct PyMT {
  uint32_t* mt;
  uint32_t* pos;
  uint32_t next() {
    if (*pos >= 624) {
      for (int i = 0; i < 624; ++i) {
        const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
        mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      *pos = 0;
    }
    uint32_t y = mt[(*pos)++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  uint64_t randbelow(uint64_t m) {
    int k = 0;
    for (uint64_t t = m; t; t >>= 1) ++k;
    for (;;) {
      const uint64_t r = next() >> (32 - k);
      if (r < m) return r;
    }
  }
};
}  // namespace

int g2v_py_shuffle_range(uint32_t* state624, uint32_t* pos, int64_t* x, int64_t n) {
  if (n > 0 && !x) return G2V_EINVAL;
  for (int64_t i = 0; i < n; ++i) x[i] = i;
  return g2v_py_shuffle(state624, pos, x, n);
}

int g2v_py_shuffle(uint32_t* state624, uint32_t* pos, int64_t* x, int64_t n) {
  if (!state624 || !pos || (n > 0 && !x)) return G2V_EINVAL;
  if (n > ((int64_t)1 << 32)) return G2V_ERANGE;
  PyMT r{state624, pos};
  // same swaps in the same order; the j of a block are drawn first so the
  // random x[j] lines can be prefetched ahead of their swap
  constexpr int kB = 4096, kAhead = 24;
  std::vector<int64_t> js(kB);
  for (int64_t hi = n - 1; hi >= 1; hi -= kB) {
    const int64_t cnt = std::min<int64_t>(kB, hi);
    for (int64_t k = 0; k < cnt; ++k) js[(size_t)k] = (int64_t)r.randbelow((uint64_t)(hi - k + 1));
    for (int64_t k = 0; k < cnt; ++k) {
      if (k + kAhead < cnt) __builtin_prefetch(x + js[(size_t)(k + kAhead)], 1);
      std::swap(x[hi - k], x[js[(size_t)k]]);
    }
  }
  return G2V_OK;
}

}  // extern "C"
