// g2v_export.cpp -- text exporters of the trained tables.
//
// Both text formats the reference's consumers read print every float32 as
// numpy's str(np.float32(v)):
//   .txt      src/generateMatrix.py:18-24   word '\t' (str(v) ' ')*D '\n'
//   _w2v.txt  [ext] save_word2vec_format    word ' ' join(' ', str(v))  '\n'
// In Python that is ~5 s of Dragon4 + string building per file at C2 (4.9 M
// values), repeated for both files in each of gene2vec.py's 10 iterations.
// Here: std::to_chars shortest round-trip digits, re-laid out with numpy's
// scalar rules (positional for 1e-4 <= |v| < 1e16 and 0, else scientific with
// a >= 2-digit exponent; 'nan', 'inf', '-0.0'), rows formatted in parallel.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <charconv>
#include <string>
#include <thread>
#include <vector>

#include "g2v.h"
#include "g2v_internal.h"

namespace {

// numpy str(np.float32(v)) into p (>= 32 bytes); returns the length
int fmt_np_f32(float v, char* p) {
  if (isnan(v)) {
    memcpy(p, "nan", 3);
    return 3;
  }
  if (isinf(v)) {
    if (v < 0) {
      memcpy(p, "-inf", 4);
      return 4;
    }
    memcpy(p, "inf", 3);
    return 3;
  }
  if (v == 0.0f) {
    if (signbit(v)) {
      memcpy(p, "-0.0", 4);
      return 4;
    }
    memcpy(p, "0.0", 3);
    return 3;
  }
  char b[48];
  const auto r = std::to_chars(b, b + sizeof b, v, std::chars_format::scientific);
  // b = [-]d[.ddd]e(+|-)XX
  const char* q = b;
  const char* end = r.ptr;
  int n = 0;
  const bool neg = *q == '-';
  if (neg) ++q;
  char dig[24];
  int nd = 0;
  while (q < end && *q != 'e') {
    if (*q != '.') dig[nd++] = *q;
    ++q;
  }
  int ex = 0;
  if (q < end) {  // 'e'
    ++q;
    const bool eneg = *q == '-';
    if (*q == '-' || *q == '+') ++q;
    while (q < end) ex = ex * 10 + (*q++ - '0');
    if (eneg) ex = -ex;
  }
  if (neg) p[n++] = '-';
  const double a = fabs((double)v);
  if (a >= 1e-4 && a < 1e16) {  // positional, at least one fractional digit
    if (ex >= 0) {
      for (int i = 0; i <= ex; ++i) p[n++] = i < nd ? dig[i] : '0';
      p[n++] = '.';
      if (nd > ex + 1) {
        for (int i = ex + 1; i < nd; ++i) p[n++] = dig[i];
      } else {
        p[n++] = '0';
      }
    } else {
      p[n++] = '0';
      p[n++] = '.';
      for (int i = 0; i < -ex - 1; ++i) p[n++] = '0';
      for (int i = 0; i < nd; ++i) p[n++] = dig[i];
    }
  } else {  // scientific: d[.ddd]e(+|-)XX
    p[n++] = dig[0];
    if (nd > 1) {
      p[n++] = '.';
      for (int i = 1; i < nd; ++i) p[n++] = dig[i];
    }
    p[n++] = 'e';
    p[n++] = ex < 0 ? '-' : '+';
    const int ae = ex < 0 ? -ex : ex;
    if (ae >= 100) p[n++] = (char)('0' + ae / 100);
    p[n++] = (char)('0' + (ae / 10) % 10);
    p[n++] = (char)('0' + ae % 10);
  }
  return n;
}

}  // namespace

extern "C" int g2v_format_f32(const float* x, int64_t n, char* out, int64_t cap,
                              int64_t* written) {
  if ((!x && n) || !written || (!out && cap) || n < 0)
    return g2v::set_error(G2V_EINVAL, "g2v_format_f32: bad arguments");
  int64_t w = 0;
  char tmp[48];
  for (int64_t i = 0; i < n; ++i) {
    const int len = fmt_np_f32(x[i], tmp);
    if (w + len + 1 > cap) return g2v::set_error(G2V_ERANGE, "g2v_format_f32: buffer too small");
    memcpy(out + w, tmp, len);
    w += len;
    out[w++] = '\n';
  }
  *written = w;
  return G2V_OK;
}

extern "C" int g2v_format_rows(const float* vectors, int64_t ld, int32_t D, const int64_t* rows,
                               int64_t n_rows, const char* words, const int64_t* word_off,
                               int32_t style, char* out, int64_t cap, int64_t* written) {
  if (!vectors || !words || !word_off || !written || D < 0 || n_rows < 0 || ld < D ||
      (style != G2V_TXT_MATRIX && style != G2V_TXT_W2V))
    return g2v::set_error(G2V_EINVAL, "g2v_format_rows: bad arguments");
  const char wsep = style == G2V_TXT_MATRIX ? '\t' : ' ';
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const int nt = (int)std::min<int64_t>(std::min(hw, 32u), std::max<int64_t>(1, n_rows / 256));
  std::vector<std::string> part((size_t)nt);
  auto work = [&](int t) {
    const int64_t r0 = n_rows * t / nt, r1 = n_rows * (t + 1) / nt;
    std::string& s = part[(size_t)t];
    s.reserve((size_t)((r1 - r0) * (16 * (int64_t)D + 32)));
    char tmp[48];
    for (int64_t k = r0; k < r1; ++k) {
      const int64_t r = rows ? rows[k] : k;
      s.append(words + word_off[k], (size_t)(word_off[k + 1] - word_off[k]));
      s.push_back(wsep);
      const float* v = vectors + r * ld;
      for (int32_t j = 0; j < D; ++j) {
        const int len = fmt_np_f32(v[j], tmp);
        s.append(tmp, (size_t)len);
        if (style == G2V_TXT_MATRIX || j + 1 < D) s.push_back(' ');
      }
      s.push_back('\n');
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& t : th) t.join();
  int64_t total = 0;
  for (auto& s : part) total += (int64_t)s.size();
  *written = total;
  if (!out) return G2V_OK;  // size query
  if (total > cap)
    return g2v::set_error(G2V_ERANGE, "g2v_format_rows: buffer of " + std::to_string(cap) +
                                          " bytes < " + std::to_string(total));
  int64_t w = 0;
  for (auto& s : part) {
    memcpy(out + w, s.data(), s.size());
    w += (int64_t)s.size();
  }
  return G2V_OK;
}
