// g2v_device.h -- device helpers shared by the kernel translation units
// (LCG jump-ahead, bucketed bisect, wave reductions, buffer-resource loads).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "g2v_internal.h"

namespace g2v {

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t lcg_step(uint64_t s) {
  return (s * 25214903917ULL + 11ULL) & kLcgMask;
}

// state after n LCG steps: two table lookups (n = lo + 2048*hi)
__device__ __forceinline__ uint64_t lcg_jump(uint64_t s, uint32_t n, const LcgJump& j) {
  const uint32_t lo = n & (kJumpTab - 1), hi = n >> kJumpBits;
  s = (j.a_lo[lo] * s + j.c_lo[lo]) & kLcgMask;
  s = (j.a_hi[hi] * s + j.c_hi[hi]) & kLcgMask;
  return s;
}

// any n >= 0: whole 2**22-step strides first (only a single sentence far
// longer than batch_words, heavily downsampled, draws that many)
__device__ __forceinline__ uint64_t lcg_jump_big(uint64_t s, uint64_t n, const LcgJump& j) {
  while (n >= kMaxJump) {
    s = lcg_step(lcg_jump(s, kMaxJump - 1, j));
    n -= kMaxJump;
  }
  return lcg_jump(s, (uint32_t)n, j);
}

// bisect_left(cum, x, 0, V) restricted to the bucket that holds x
__device__ __forceinline__ int32_t bisect_bucket(const uint32_t* __restrict__ cum,
                                                 const int32_t* __restrict__ bkt, int32_t V,
                                                 uint32_t x) {
  const uint32_t b = x >> kBucketShift;
  int32_t lo = bkt[b], hi = bkt[b + 1];
  if (hi > V - 1) hi = V - 1;
  while (hi > lo) {
    const int32_t mid = (lo + hi) >> 1;
    if (cum[mid] >= x) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// one gensim negative draw: t = bisect_left(cum, (nr>>16) % cum[-1]); nr advances
__device__ __forceinline__ int32_t draw_negative(uint64_t& nr, const uint32_t* __restrict__ cum,
                                                 const int32_t* __restrict__ bkt, int32_t V,
                                                 uint32_t cum_last) {
  const uint32_t x = ((uint32_t)(nr >> 16)) % cum_last;
  nr = lcg_step(nr);
  return bisect_bucket(cum, bkt, V, x);
}

template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int* sh, int& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[wid] = x;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const int t = sh[w];
    base += (w < wid) ? t : 0;
    tot += t;
  }
  __syncthreads();
  total = tot;
  return base + x - v;
}

__device__ __forceinline__ int64_t sent_start(const SampleArgs& a, int64_t s) {
  return a.sent_len > 0 ? s * a.sent_len : a.sent_off[s];
}


// ---------------------------------------------------------------------------
// wave reductions (64 lanes)
// ---------------------------------------------------------------------------
template <int N>
struct Pow2 {
  static constexpr int v = (N <= 1) ? 1 : 2 * Pow2<(N + 1) / 2>::v;
};
template <>
struct Pow2<1> {
  static constexpr int v = 1;
};

__device__ __forceinline__ double shfl_xor_d(double v, int m) {
  const long long b = __double_as_longlong(v);
  const int lo = __shfl_xor((int)(b & 0xffffffffLL), m, 64);
  const int hi = __shfl_xor((int)(b >> 32), m, 64);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double wave_allreduce_d(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += shfl_xor_d(v, m);
  return v;
}

// Sum NT per-lane values over the 64 lanes: value-halving xor butterfly (each
// exchange step halves the values a lane carries), then a plain butterfly on
// the last one; the NT totals end up wave-uniform.
template <int NT>
__device__ __forceinline__ void wave_reduce_multi(const double (&in)[NT], double (&out)[NT],
                                                  int lane) {
  constexpr int P = Pow2<NT>::v;
  static_assert(P <= 64, "too many values");
  double x[P];
#pragma unroll
  for (int i = 0; i < P; ++i) x[i] = (i < NT) ? in[i] : 0.0;
  int m = 32;
#pragma unroll
  for (int h = P / 2; h >= 1; h >>= 1) {
    const bool up = (lane & m) != 0;
#pragma unroll
    for (int i = 0; i < h; ++i) {
      const double send = up ? x[i] : x[i + h];
      const double keep = up ? x[i + h] : x[i];
      x[i] = keep + shfl_xor_d(send, m);
    }
    m >>= 1;
  }
#pragma unroll
  for (; m >= 1; m >>= 1) x[0] += shfl_xor_d(x[0], m);
  // value v lives in lanes whose halving bits spell v
#pragma unroll
  for (int v = 0; v < NT; ++v) {
    int src = 0, mm = 32;
#pragma unroll
    for (int h = P / 2; h >= 1; h >>= 1) {
      if (v & h) src += mm;
      mm >>= 1;
    }
    out[v] = readlane_d(x[0], src);
  }
}

constexpr int kPolPlain = 0;
constexpr int kPolWt = 1;
constexpr int kPolWtRd = 2;

template <int POL>
struct Pol {
  static constexpr int ld = (POL == kPolWtRd) ? 16 : 0;  // sc1
  static constexpr int st = (POL == kPolPlain) ? 0 : 16;  // sc1
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0,
                                           (int)(bytes > 0x7fffffff ? 0x7fffffff : bytes),
                                           0x00020000);
}

template <int AUX>
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, int off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
  float4 o;
  o.x = __uint_as_float(v[0]);
  o.y = __uint_as_float(v[1]);
  o.z = __uint_as_float(v[2]);
  o.w = __uint_as_float(v[3]);
  return o;
}

template <int AUX>
__device__ __forceinline__ void bstore4(__amdgpu_buffer_rsrc_t r, int off, float4 v) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  u4 u;
  u[0] = __float_as_uint(v.x);
  u[1] = __float_as_uint(v.y);
  u[2] = __float_as_uint(v.z);
  u[3] = __float_as_uint(v.w);
  __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, AUX);
}

template <int AUX>
__device__ __forceinline__ float bload1(__amdgpu_buffer_rsrc_t r, int off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, AUX));
}

__device__ __forceinline__ double dot4(const float4& a, const float4& b, double s) {
  s = fma((double)a.x, (double)b.x, s);
  s = fma((double)a.y, (double)b.y, s);
  s = fma((double)a.z, (double)b.z, s);
  s = fma((double)a.w, (double)b.w, s);
  return s;
}

}  // namespace g2v
