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

// Cross-lane exchanges without LDS (no ds_bpermute): gfx950's
// v_permlane32_swap / v_permlane16_swap for the lane masks 32 and 16, DPP
// (row_ror:8, row_half_mirror, quad_perm) inside a row for 8, 4, 2, 1.  The
// partner of lane l at mask m is l^m, except m = 4 where row_half_mirror pairs
// l with l^7 (an involution that also flips bit 2: every butterfly below only
// needs "partner differs in bit m, later stages cover the rest").
__device__ __forceinline__ uint32_t lo32(double v) {
  return (uint32_t)(__double_as_longlong(v) & 0xffffffffLL);
}
__device__ __forceinline__ uint32_t hi32(double v) {
  return (uint32_t)((unsigned long long)__double_as_longlong(v) >> 32);
}
__device__ __forceinline__ double mk_d(uint32_t lo, uint32_t hi) {
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

template <int M>
struct DppCtrl;
template <>
struct DppCtrl<8> { static constexpr int v = 0x128; };  // row_ror:8   -> l ^ 8
template <>
struct DppCtrl<4> { static constexpr int v = 0x141; };  // row_half_mirror -> l ^ 7
template <>
struct DppCtrl<2> { static constexpr int v = 0x4e; };   // quad_perm [2,3,0,1] -> l ^ 2
template <>
struct DppCtrl<1> { static constexpr int v = 0xb1; };   // quad_perm [1,0,3,2] -> l ^ 1

template <int M>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)lo32(v), DppCtrl<M>::v, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)hi32(v), DppCtrl<M>::v, 0xf, 0xf, false);
  return mk_d((uint32_t)lo, (uint32_t)hi);
}

// Lanes with bit M clear get a + partner's a, lanes with bit M set get
// b + partner's b (one butterfly step carrying two values, keeping one).
template <int M>
__device__ __forceinline__ double xchg_pair(double a, double b, int lane) {
  if constexpr (M == 32 || M == 16) {
    // swap the upper 32 lanes of a with the lower 32 of b (M = 32), or the odd
    // 16-lane rows of a with the even rows of b (M = 16): afterwards the two
    // registers hold, lane for lane, the two addends of the wanted sum
    auto slo = M == 32 ? __builtin_amdgcn_permlane32_swap(lo32(a), lo32(b), false, false)
                       : __builtin_amdgcn_permlane16_swap(lo32(a), lo32(b), false, false);
    auto shi = M == 32 ? __builtin_amdgcn_permlane32_swap(hi32(a), hi32(b), false, false)
                       : __builtin_amdgcn_permlane16_swap(hi32(a), hi32(b), false, false);
    return mk_d(slo[0], shi[0]) + mk_d(slo[1], shi[1]);
  } else {
    const bool up = (lane & M) != 0;
    const double send = up ? a : b;
    const double keep = up ? b : a;
    return keep + dpp_d<M>(send);
  }
}

// every lane: x + partner's x at mask M
template <int M>
__device__ __forceinline__ double xsum_d(double x) {
  if constexpr (M == 32 || M == 16) {
    return xchg_pair<M>(x, x, 0);
  } else {
    return x + dpp_d<M>(x);
  }
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double wave_allreduce_d(double v) {
  v = xsum_d<32>(v);
  v = xsum_d<16>(v);
  v = xsum_d<8>(v);
  v = xsum_d<4>(v);
  v = xsum_d<2>(v);
  v = xsum_d<1>(v);
  return v;
}

// one value-halving butterfly stage over the masks 32, 16, ..., 1 (index S)
template <int S, int H, int P>
__device__ __forceinline__ void halve_stage(double (&x)[P], int lane) {
  constexpr int M = 32 >> S;
#pragma unroll
  for (int i = 0; i < H; ++i) x[i] = xchg_pair<M>(x[i], x[i + H], lane);
}

template <int S, int P>
__device__ __forceinline__ void halve_all(double (&x)[P], int lane) {
  constexpr int H = P >> (S + 1);  // values kept after this stage
  if constexpr (H >= 1) {
    halve_stage<S, H, P>(x, lane);
    halve_all<S + 1, P>(x, lane);
  } else if constexpr (S <= 5) {
    x[0] = xsum_d<(32 >> S)>(x[0]);
    halve_all<S + 1, P>(x, lane);
  }
}

// Sum NT per-lane values over the 64 lanes: value-halving butterfly (each
// stage exchanges half of the values a lane carries and keeps the other
// half), then a plain butterfly on the last one; the NT totals end up
// wave-uniform.
template <int NT>
__device__ __forceinline__ void wave_reduce_multi(const double (&in)[NT], double (&out)[NT],
                                                  int lane) {
  constexpr int P = Pow2<NT>::v;
  static_assert(P <= 64, "too many values");
  double x[P];
#pragma unroll
  for (int i = 0; i < P; ++i) x[i] = (i < NT) ? in[i] : 0.0;
  halve_all<0, P>(x, lane);
  // value v lives in lanes whose halving bits spell v: bit h of v <-> lane
  // bit (32 >> stage)
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
