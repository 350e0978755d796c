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
#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <new>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "g2v.h"

namespace {

// byte classes of the tokenizer: 0 word byte, 1 str.split() separator,
// 2 line terminator ('\n' / '\r'), 3 byte undefined in windows-1252 (Python's
// decoder raises UnicodeDecodeError)
struct ByteClass {
  uint8_t c[256];
  constexpr ByteClass() : c() {
    for (int i = 0; i < 256; ++i) c[i] = 0;
    c[' '] = 1;
    for (int i = 0x09; i <= 0x0d; ++i) c[i] = 1;
    for (int i = 0x1c; i <= 0x1f; ++i) c[i] = 1;
    c[0xa0] = 1;
    c['\n'] = 2;
    c['\r'] = 2;
    c[0x81] = c[0x8d] = c[0x8f] = c[0x90] = c[0x9d] = 3;
  }
};
constexpr ByteClass kClass{};

inline uint64_t hash_bytes(const unsigned char* p, size_t n) {
  uint64_t h = 0x9e3779b97f4a7c15ull ^ (uint64_t)n;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    h = (h ^ v) * 0xbf58476d1ce4e5b9ull;
    h ^= h >> 31;
    p += 8;
    n -= 8;
  }
  uint64_t v = 0;
  for (size_t i = 0; i < n; ++i) v |= (uint64_t)p[i] << (8 * i);
  h = (h ^ v) * 0x94d049bb133111ebull;
  h ^= h >> 29;
  h *= 0xbf58476d1ce4e5b9ull;
  return h ^ (h >> 32);
}

struct Chunk {  // a line-aligned piece of one file
  const char* p = nullptr;
  size_t n = 0;
  std::vector<int32_t> tok;              // local ids
  int64_t lines = 0;                     // sentences in the chunk
  int64_t fixed = -1;                    // their common length while len is empty (-1: none yet)
  std::vector<int64_t> len;              // sentence lengths, once two lengths differ
  std::vector<std::string_view> words;   // local id -> bytes (views into the file buffer)
  std::vector<uint64_t> hash;            // local id -> hash_bytes(word)
  std::vector<int64_t> cnt;              // local counts
  int err = 0;
  void end_line(int64_t ntok) {
    if (len.empty() && (fixed < 0 || fixed == ntok)) {
      fixed = ntok;  // pair files: every line 2 tokens, nothing stored
    } else {
      if (len.empty()) len.assign((size_t)lines, fixed);
      len.push_back(ntok);
    }
    ++lines;
  }
  int64_t length(int64_t i) const { return len.empty() ? fixed : len[(size_t)i]; }
};

// open-addressing word -> id table (linear probing, load <= 1/2).  A slot
// holds the hash, the length and the first 16 bytes of its word, so a lookup
// of a gene name (almost always <= 16 bytes) touches one 32-B slot.
struct WordTable {
  struct Slot {
    uint64_t h;
    int32_t id;  // -1 = empty
    uint32_t len;
    char pfx[16];
  };
  std::vector<Slot> slot;
  uint64_t mask = 0;
  explicit WordTable(size_t cap = 1 << 16) : slot(cap, Slot{0, -1, 0, {}}), mask(cap - 1) {}
  // id of w, or the slot index (encoded as -1 - slot) where it would go
  template <class Words>
  int64_t find(const Words& words, std::string_view w, uint64_t h) const {
    uint64_t k = h & mask;
    for (;;) {
      const Slot& e = slot[k];
      if (e.id < 0) return -1 - (int64_t)k;
      if (e.h == h && e.len == w.size() &&
          (w.size() <= 16 ? memcmp(e.pfx, w.data(), w.size()) == 0 : words[e.id] == w))
        return e.id;
      k = (k + 1) & mask;
    }
  }
  // fill the slot find() returned for a new word; grows at load 1/2
  void insert(int64_t where, std::string_view w, uint64_t h, int32_t id) {
    Slot& e = slot[(size_t)(-1 - where)];
    e.h = h;
    e.id = id;
    e.len = (uint32_t)w.size();
    memcpy(e.pfx, w.data(), std::min<size_t>(16, w.size()));
    if ((size_t)id * 2 + 2 > slot.size()) {
      std::vector<Slot> s2(slot.size() * 2, Slot{0, -1, 0, {}});
      const uint64_t m2 = s2.size() - 1;
      for (const Slot& o : slot) {
        if (o.id < 0) continue;
        uint64_t k = o.h & m2;
        while (s2[k].id >= 0) k = (k + 1) & m2;
        s2[k] = o;
      }
      slot.swap(s2);
      mask = m2;
    }
  }
};

void tokenize(Chunk& c) {
  WordTable tab;
  const unsigned char* s = (const unsigned char*)c.p;
  const size_t n = c.n;
  c.tok.reserve(n / 6 + 16);
  size_t i = 0;
  while (i < n) {
    // one line: up to '\n', '\r\n' or '\r'
    int64_t ntok = 0;
    for (;;) {
      while (i < n && kClass.c[s[i]] == 1) ++i;
      if (i >= n || kClass.c[s[i]] == 2) break;
      const size_t b = i;
      uint8_t cls;
      while (i < n && ((cls = kClass.c[s[i]]) == 0 || cls == 3)) {
        c.err |= cls == 3;
        ++i;
      }
      const std::string_view w((const char*)s + b, i - b);
      const uint64_t h = hash_bytes(s + b, i - b);
      int64_t id = tab.find(c.words, w, h);
      if (id < 0) {
        tab.insert(id, w, h, (int32_t)c.words.size());
        id = (int64_t)c.words.size();
        c.words.push_back(w);
        c.hash.push_back(h);
        c.cnt.push_back(0);
      }
      c.cnt[(size_t)id]++;
      c.tok.push_back((int32_t)id);
      ++ntok;
    }
    c.end_line(ntok);
    if (i < n) {  // consume the line terminator
      if (s[i] == '\r' && i + 1 < n && s[i + 1] == '\n') i += 2;
      else ++i;
    }
  }
}

template <class Fn>
void parallel_for(size_t n, int threads, Fn&& fn) {
  const int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads, n));
  std::atomic_size_t next{0};
  auto body = [&]() {
    for (size_t k; (k = next.fetch_add(1)) < n;) fn(k);
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(body);
  body();
  for (auto& t : th) t.join();
}

}  // namespace

struct g2v_corpus {
  std::vector<Chunk> chunks;                   // tokens in chunk-local ids
  std::vector<std::vector<int32_t>> remap;     // chunk-local id -> global id
  std::vector<int64_t> tbase, sbase;           // token / sentence offset of each chunk
  int64_t fixed_len = -1;                      // common sentence length, -1 = ragged
  int threads = 8;
  std::vector<std::string> words;              // global id -> bytes (windows-1252)
  std::vector<int64_t> counts;
};

extern "C" {

int g2v_corpus_read(const char* const* paths, int n_paths, int n_threads, g2v_corpus** out) {
  if (!out || (n_paths > 0 && !paths) || n_paths < 0) return G2V_EINVAL;
  *out = nullptr;
  std::unique_ptr<g2v_corpus> cp(new (std::nothrow) g2v_corpus());
  if (!cp) return G2V_ENOMEM;
  const int threads = n_threads > 0 ? n_threads : 8;
  cp->threads = threads;
  // files mapped read-only from the page cache (no copy, no zero-filled
  // buffer); unmapped when the read returns (words are copied out, tokens are
  // ids)
  struct Map {
    const char* p = nullptr;
    size_t n = 0;
    ~Map() {
      if (p && n) munmap(const_cast<char*>(p), n);
    }
  };
  std::vector<Map> maps(n_paths);
  for (int f = 0; f < n_paths; ++f) {
    const int fd = open(paths[f], O_RDONLY);
    struct stat st;
    if (fd < 0 || fstat(fd, &st) != 0) {
      if (fd >= 0) close(fd);
      return G2V_EINVAL;
    }
    maps[f].n = (size_t)st.st_size;
    if (maps[f].n) {
      void* m = mmap(nullptr, maps[f].n, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
      if (m == MAP_FAILED) {
        maps[f].n = 0;
        close(fd);
        return G2V_EINVAL;
      }
      maps[f].p = static_cast<const char*>(m);
    }
    close(fd);
  }
  // line-aligned chunks of ~16 MiB, in file order
  std::vector<Chunk>& chunks = cp->chunks;
  const size_t target = (size_t)16 << 20;
  for (int f = 0; f < n_paths; ++f) {
    const char* buf = maps[f].p;
    const size_t n = maps[f].n;
    size_t b = 0;
    while (b < n) {
      size_t e = std::min(n, b + target);
      while (e < n && buf[e - 1] != '\n' && buf[e - 1] != '\r') ++e;
      // never split a "\r\n" pair
      if (e < n && buf[e - 1] == '\r' && buf[e] == '\n') ++e;
      Chunk c;
      c.p = buf + b;
      c.n = e - b;
      chunks.push_back(std::move(c));
      b = e;
    }
  }
  parallel_for(chunks.size(), threads, [&](size_t k) { tokenize(chunks[k]); });
  for (auto& c : chunks)
    if (c.err) return G2V_EINVAL;  // UnicodeDecodeError in the reference
  // global ids in first-occurrence order = chunk order, then local order
  // (sequential over each chunk's vocabulary only); the token remap itself
  // runs in g2v_corpus_export, straight into the caller's buffer
  WordTable gtab(1 << 16);
  std::vector<std::string_view> gwords;
  cp->remap.resize(chunks.size());
  cp->tbase.assign(chunks.size() + 1, 0);
  cp->sbase.assign(chunks.size() + 1, 0);
  int64_t fixed = -2;  // -2: no sentence yet
  for (size_t k = 0; k < chunks.size(); ++k) {
    Chunk& c = chunks[k];
    std::vector<int32_t>& rm = cp->remap[k];
    rm.resize(c.words.size());
    for (size_t l = 0; l < c.words.size(); ++l) {
      int64_t g = gtab.find(gwords, c.words[l], c.hash[l]);
      if (g < 0) {
        gtab.insert(g, c.words[l], c.hash[l], (int32_t)gwords.size());
        g = (int64_t)gwords.size();
        gwords.push_back(c.words[l]);
        cp->counts.push_back(0);
      }
      rm[l] = (int32_t)g;
      cp->counts[(size_t)g] += c.cnt[l];
    }
    // views into the mapped files are not kept past the read
    c.p = nullptr;
    std::vector<uint64_t>().swap(c.hash);
    std::vector<int64_t>().swap(c.cnt);
    cp->tbase[k + 1] = cp->tbase[k] + (int64_t)c.tok.size();
    cp->sbase[k + 1] = cp->sbase[k] + c.lines;
    if (c.lines) {
      const int64_t cf = c.len.empty() ? c.fixed : -1;
      fixed = (fixed == -2 || fixed == cf) ? cf : -1;
    }
  }
  cp->fixed_len = fixed == -2 ? -1 : fixed;
  cp->words.reserve(gwords.size());
  for (auto& w : gwords) cp->words.emplace_back(w);
  for (auto& c : chunks) std::vector<std::string_view>().swap(c.words);
  *out = cp.release();
  return G2V_OK;
}

int g2v_corpus_info(const g2v_corpus* c, int64_t* n_tokens, int64_t* n_sent, int64_t* n_words,
                    int64_t* word_bytes) {
  if (!c) return G2V_EINVAL;
  if (n_tokens) *n_tokens = c->tbase.empty() ? 0 : c->tbase.back();
  if (n_sent) *n_sent = c->sbase.empty() ? 0 : c->sbase.back();
  if (n_words) *n_words = (int64_t)c->words.size();
  if (word_bytes) {
    int64_t b = 0;
    for (auto& w : c->words) b += (int64_t)w.size();
    *word_bytes = b;
  }
  return G2V_OK;
}

int g2v_count_lines(const char* const* paths, int n_paths, int n_threads, int64_t* out) {
  if (!out || (n_paths > 0 && !paths) || n_paths < 0) return G2V_EINVAL;
  *out = 0;
  const int threads = n_threads > 0 ? n_threads : 8;
  std::atomic<int64_t> total{0};
  for (int f = 0; f < n_paths; ++f) {
    const int fd = open(paths[f], O_RDONLY);
    struct stat st;
    if (fd < 0 || fstat(fd, &st) != 0) {
      if (fd >= 0) close(fd);
      return G2V_EINVAL;
    }
    const size_t n = (size_t)st.st_size;
    if (n == 0) {
      close(fd);
      continue;
    }
    void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return G2V_EINVAL;
    const unsigned char* b = static_cast<const unsigned char*>(m);
    // universal newlines, as the tokenizer splits: '\n', "\r\n" and a lone
    // '\r' end a line; an unterminated last line is a line too
    constexpr size_t kPiece = (size_t)16 << 20;
    const size_t pieces = (n + kPiece - 1) / kPiece;
    parallel_for(pieces, threads, [&](size_t k) {
      const size_t lo = k * kPiece, hi = std::min(n, lo + kPiece);
      int64_t c = 0;
      for (size_t i = lo; i < hi; ++i)
        c += (b[i] == '\n') + (b[i] == '\r' && (i + 1 == n || b[i + 1] != '\n'));
      total += c;
    });
    if (b[n - 1] != '\n' && b[n - 1] != '\r') total += 1;
    munmap(m, n);
  }
  *out = total.load();
  return G2V_OK;
}

int g2v_corpus_sent_len(const g2v_corpus* c, int64_t* len) {
  if (!c || !len) return G2V_EINVAL;
  *len = c->fixed_len;
  return G2V_OK;
}

// tokens[n_tokens], sent_off[n_sent+1], counts[n_words], words as concatenated
// bytes + word_off[n_words+1]; any pointer may be NULL
int g2v_corpus_export(const g2v_corpus* c, int32_t* tokens, int64_t* sent_off, int64_t* counts,
                      char* words, int64_t* word_off) {
  if (!c) return G2V_EINVAL;
  if (sent_off) sent_off[0] = 0;
  if (tokens || sent_off)
    parallel_for(c->chunks.size(), c->threads, [&](size_t k) {
      const Chunk& ch = c->chunks[k];
      if (tokens) {
        const int32_t* rm = c->remap[k].data();
        int32_t* dst = tokens + c->tbase[k];
        for (size_t i = 0; i < ch.tok.size(); ++i) dst[i] = rm[ch.tok[i]];
      }
      if (sent_off) {
        int64_t o = c->tbase[k];
        int64_t* od = sent_off + c->sbase[k] + 1;
        for (int64_t i = 0; i < ch.lines; ++i) od[i] = (o += ch.length(i));
      }
    });
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

int g2v_pairs_permute(const int32_t* tok, int64_t n_pairs, const int64_t* perm,
                      int32_t* out_tok) {
  if (n_pairs < 0 || (n_pairs > 0 && (!tok || !perm || !out_tok))) return G2V_EINVAL;
  // one 8-byte random read per pair (the CSR form reads two offsets per pair
  // in each of its two passes); output written sequentially
  const int nt = (int)std::min<int64_t>(16, std::max<int64_t>(1, n_pairs >> 16));
  const uint64_t* src = reinterpret_cast<const uint64_t*>(tok);
  uint64_t* dst = reinterpret_cast<uint64_t*>(out_tok);
  std::atomic<bool> bad{false};
  std::vector<std::thread> th;
  auto fn = [&](int t) {
    const int64_t a = n_pairs * t / nt, b = n_pairs * (t + 1) / nt;
    constexpr int64_t kAhead = 16;
    for (int64_t i = a; i < b; ++i) {
      if (i + kAhead < b) {
        const int64_t q = perm[i + kAhead];
        if (q >= 0 && q < n_pairs) __builtin_prefetch(src + q);
      }
      const int64_t p = perm[i];
      if (p < 0 || p >= n_pairs) {
        bad = true;
        return;
      }
      uint64_t v;
      memcpy(&v, src + p, 8);
      dst[i] = v;
    }
  };
  for (int t = 1; t < nt; ++t) th.emplace_back(fn, t);
  fn(0);
  for (auto& x : th) x.join();
  return bad ? G2V_EINVAL : G2V_OK;
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
  uint64_t randbelow(uint64_t m) {  // 2 <= m < 2^32
    const int k = 64 - __builtin_clzll(m);
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

int g2v_py_shuffle_skip(uint32_t* state624, uint32_t* pos, int64_t n) {
  if (!state624 || !pos) return G2V_EINVAL;
  if (n >= ((int64_t)1 << 32)) return G2V_ERANGE;
  PyMT r{state624, pos};
  for (int64_t i = n - 1; i >= 1; --i) (void)r.randbelow((uint64_t)(i + 1));
  return G2V_OK;
}

int g2v_py_shuffle(uint32_t* state624, uint32_t* pos, int64_t* x, int64_t n) {
  if (!state624 || !pos || (n > 0 && !x)) return G2V_EINVAL;
  if (n >= ((int64_t)1 << 32)) return G2V_ERANGE;  // _randbelow(2^32) draws 2 words
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
