// g2v_host.cpp -- host-native helpers of libg2v.so (no device work).
//
//   lcg_jump_tables      affine powers of gensim's 48-bit LCG
//                        ([ext] word2vec_inner.pyx random_int32) for O(1)
//                        jump-ahead on the device
//   g2v_seeded_vectors   [ext] Word2VecTrainables.seeded_vector for all rows:
//                        numpy RandomState(seed).rand(D) (MT19937 init_genrand +
//                        53-bit random_sample) reimplemented natively
//   g2v_count_ids        [ext] scan_vocab over pre-hashed integer ids
#include <stdint.h>
#include <string.h>

#include <string>

#include "g2v.h"
#include "g2v_internal.h"

namespace g2v {

void lcg_jump_tables(uint64_t* a_lo, uint64_t* c_lo, uint64_t* a_hi, uint64_t* c_hi) {
  const uint64_t A = 25214903917ULL, C = 11ULL;
  // x_{n+1} = A x_n + C: (a_n, c_n) with x_n = a_n x_0 + c_n
  uint64_t a = 1, c = 0;
  for (int n = 0; n < kJumpTab; ++n) {
    a_lo[n] = a;
    c_lo[n] = c;
    a = (A * a) & kLcgMask;
    c = (A * c + C) & kLcgMask;
  }
  // (a, c) now is the 2048-step map; powers of it for the high table
  const uint64_t a2048 = a, c2048 = c;
  uint64_t ah = 1, ch = 0;
  for (int n = 0; n < kJumpTab; ++n) {
    a_hi[n] = ah;
    c_hi[n] = ch;
    const uint64_t na = (a2048 * ah) & kLcgMask;
    const uint64_t nc = (a2048 * ch + c2048) & kLcgMask;
    ah = na;
    ch = nc;
  }
}

namespace {
struct MT19937 {
  uint32_t mt[624];
  int pos = 624;
  explicit MT19937(uint32_t s) {
    mt[0] = s;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
  }
  uint32_t next() {
    if (pos >= 624) {
      for (int i = 0; i < 624; ++i) {
        const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
        mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      pos = 0;
    }
    uint32_t y = mt[pos++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  double random_sample() {  // numpy legacy random_double
    const uint32_t a = next() >> 5, b = next() >> 6;
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }
};
}  // namespace

}  // namespace g2v

extern "C" {

int g2v_seeded_vectors(const uint32_t* seeds, int64_t n_rows, int32_t dim, float* out) {
  if ((!seeds || !out) && n_rows > 0) return G2V_EINVAL;
  if (dim <= 0 || n_rows < 0) return G2V_EINVAL;
  for (int64_t i = 0; i < n_rows; ++i) {
    g2v::MT19937 rs(seeds[i]);
    float* row = out + i * dim;
    for (int32_t k = 0; k < dim; ++k) row[k] = (float)((rs.random_sample() - 0.5) / (double)dim);
  }
  return G2V_OK;
}

int g2v_count_ids(const int32_t* ids, int64_t n, int32_t V, int64_t* counts, int64_t* first) {
  if (V <= 0 || n < 0 || !counts || (!ids && n > 0)) return G2V_EINVAL;
  memset(counts, 0, sizeof(int64_t) * V);
  if (first)
    for (int32_t i = 0; i < V; ++i) first[i] = -1;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t w = ids[i];
    if (w < 0 || w >= V) return G2V_ERANGE;
    if (first && counts[w] == 0) first[w] = i;
    counts[w]++;
  }
  return G2V_OK;
}

}  // extern "C"
