// g2v_kernels.hip -- CDNA4 (gfx950) kernels of the Gene2vec SGNS hot path.
//
// Replaces gensim 3.4.0's Cython/C inner loop ([ext] word2vec_inner.pyx:
// train_batch_sg + fast_sentence_sg_neg + init())
// that src/gene2vec.py:70,87 drives.  Three kernels per segment of jobs:
//
//   k_job_sample<false>  one workgroup per gensim job: OOV skip + frequent-word
//                        downsampling with the job's 48-bit LCG (jumped ahead,
//                        not iterated), window-1 example count
//   k_scan_jobs          exclusive scan of per-job example counts
//   k_job_sample<true>   same pass again, now writing one record per directed
//                        example {center, input, alpha, negs[K]} with the K
//                        negatives drawn exactly as gensim draws them (LCG state
//                        = jump(seed, draws_before), bisect over cum_table
//                        accelerated by a 2^16-bucket index)
//   k_sgns<K,NV,MODE>    the update: ONE WAVE PER DIRECTED EXAMPLE, lane l owns
//                        float4 columns l (+64): 16-B row gathers from
//                        syn0/syn1neg, K+1 dots in fp64 (dsdot) reduced across the
//                        wave by a value-halving xor butterfly, LUT sigmoid from
//                        LDS, gradient + work accumulation in registers, and
//                        plain (Hogwild) float4 write-back of every touched row.
//
// Everything is memory-gather bound (0.68 flop/B): no MFMA by design.
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
// k_job_sample: one workgroup per job ([ext] train_batch_sg pre-pass)
// ---------------------------------------------------------------------------
template <bool WRITE>
__global__ __launch_bounds__(kSampleThreads) void k_job_sample(SampleArgs a) {
  __shared__ int32_t s_eff[kBatchWords];       // kept tokens, compacted
  __shared__ uint16_t s_kc[kBatchWords + 1];   // kept-before count per raw position
  __shared__ int s_scan[kSampleThreads / 64];

  const int64_t j = blockIdx.x;                // job within segment
  const int64_t jg = a.job0 + j;
  const int64_t s0 = a.job_sent[jg], s1 = a.job_sent[jg + 1];
  const int64_t tb = sent_start(a, s0);
  const int n = (int)(sent_start(a, s1) - tb);  // <= kBatchWords (host-checked)
  const uint64_t seed = a.job_seed[jg];

  int inv_base = 0, keep_base = 0;
  for (int t0 = 0; t0 < n; t0 += kSampleThreads) {
    const int t = t0 + threadIdx.x;
    const int32_t w = (t < n) ? a.tok[tb + t] : -1;
    const int inv = (w >= 0);
    int tot_inv;
    const int p = inv_base + block_excl_scan<kSampleThreads>(inv, s_scan, tot_inv);
    int keep = inv;
    if (inv && a.sample_on) {
      // gensim: drop iff sample_int < random_int32(&next_random); the p-th draw
      const uint32_t r = (uint32_t)(lcg_jump(seed, (uint32_t)p, a.jump) >> 16);
      keep = !(a.sample_int[w] < r);
    }
    int tot_keep;
    const int c = keep_base + block_excl_scan<kSampleThreads>(keep, s_scan, tot_keep);
    if (t < n) {
      s_kc[t] = (uint16_t)c;
      if (keep) s_eff[c] = w;
    }
    inv_base += tot_inv;
    keep_base += tot_keep;
  }
  if (threadIdx.x == 0) s_kc[n] = (uint16_t)keep_base;
  __syncthreads();

  const uint32_t ndraw = a.sample_on ? (uint32_t)inv_base : 0u;
  const int ns = (int)(s1 - s0);
  const float alpha = WRITE ? a.job_alpha[jg] : 0.f;
  const int64_t out_base = WRITE ? a.job_exoff[j] : 0;
  const uint32_t cum_last = a.cum[a.V - 1];
  int ex_base = 0;
  for (int q0 = 0; q0 < ns; q0 += kSampleThreads) {
    const int q = q0 + threadIdx.x;
    int e0 = 0, e1 = 0;
    if (q < ns) {
      e0 = s_kc[sent_start(a, s0 + q) - tb];
      e1 = s_kc[sent_start(a, s0 + q + 1) - tb];
    }
    const int L = e1 - e0;
    const int nex = L >= 2 ? 2 * (L - 1) : 0;  // window 1: (i,i-1),(i,i+1) in range
    int tot;
    const int eb = ex_base + block_excl_scan<kSampleThreads>(nex, s_scan, tot);
    if (WRITE && nex) {
      int e = eb;
      for (int i = e0; i < e1; ++i) {
#pragma unroll
        for (int dj = -1; dj <= 1; dj += 2) {
          const int jj = i + dj;
          if (jj < e0 || jj >= e1) continue;
          int32_t* r = a.rec + (out_base + e) * a.rec_stride;
          const int32_t center = s_eff[i];
          r[0] = center;
          r[1] = s_eff[jj];
          r[2] = __float_as_int(alpha);
          uint64_t nr = lcg_jump(seed, ndraw + (uint32_t)a.K * (uint32_t)e, a.jump);
          for (int d = 0; d < a.K; ++d) {
            const int32_t t = draw_negative(nr, a.cum, a.bkt, a.V, cum_last);
            r[3 + d] = (t == center) ? -1 : t;
          }
          ++e;
        }
      }
    }
    ex_base += tot;
  }
  if (!WRITE && threadIdx.x == 0) {
    a.job_nex[j] = ex_base;
    atomicAdd(a.counters + 0, (unsigned long long)keep_base);  // effective words
    atomicAdd(a.counters + 2, (unsigned long long)n);          // raw words
  }
}

// ---------------------------------------------------------------------------
// k_scan_jobs: exclusive scan of the per-job example counts (one workgroup)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_scan_jobs(const int32_t* __restrict__ nex, int64_t nj,
                                                    int64_t* __restrict__ off,
                                                    unsigned long long* examples_total) {
  __shared__ int s[16];
  int64_t carry = 0;
  for (int64_t b = 0; b < nj; b += 1024) {
    const int64_t i = b + threadIdx.x;
    const int v = i < nj ? nex[i] : 0;
    int tot;
    const int ex = block_excl_scan<1024>(v, s, tot);
    if (i < nj) off[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) {
    off[nj] = carry;
    atomicAdd(examples_total, (unsigned long long)carry);
  }
}

// ---------------------------------------------------------------------------
// k_explicit_records: records from host-provided (center, input, negs)
// ---------------------------------------------------------------------------
__global__ void k_explicit_records(const int32_t* __restrict__ center,
                                   const int32_t* __restrict__ input,
                                   const int32_t* __restrict__ negs, int64_t n, int K, float alpha,
                                   int rec_stride, int32_t* __restrict__ rec) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int32_t* r = rec + i * rec_stride;
  r[0] = center[i];
  r[1] = input[i];
  r[2] = __float_as_int(alpha);
  for (int d = 0; d < K; ++d) {
    const int32_t t = negs[i * K + d];
    r[3 + d] = (t == center[i]) ? -1 : t;
  }
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

// ---------------------------------------------------------------------------
// k_sgns: one wave per directed example ([ext] fast_sentence_sg_neg)
// ---------------------------------------------------------------------------
// Table traffic goes through buffer resources so every load/store carries an
// explicit cache policy (POL, compile time):
//   kPolPlain   default policy (lines stay in the issuing XCD's L2)
//   kPolWt      stores sc1 (write-through to the coherent side, line dropped
//               from the writer's L2) -- other XCDs see updates within the launch
//   kPolWtRd    kPolWt + sc1 loads
// Rows with vocabulary index < hot_rows (the most frequent genes: indices are
// sorted by descending count) are never stored: their deltas go to the memory
// side as float atomics, one 256-B contiguous wave-instruction per 64 columns,
// so concurrent updates of a hot row are summed, not lost.
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

template <int K, int NV, int MODE, int POL>
__global__ __launch_bounds__(kSgnsThreads) void k_sgns(SgnsArgs a) {
  __shared__ float s_lut[kExpTableSize];
  __shared__ float s_work[kSgnsThreads / 64][64 * 4 * NV];  // per-wave transpose buffer
  for (int i = threadIdx.x; i < kExpTableSize; i += kSgnsThreads) s_lut[i] = a.exp_table[i];
  __syncthreads();

  constexpr int NT = K + 1;
  constexpr int LA = Pol<POL>::ld, SA = Pol<POL>::st;
  constexpr int NE = NV * 4;  // element-layout columns per lane (l + 64 i)
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  int64_t gw, nw;
  if (MODE == kModeSequential) {
    if (blockIdx.x != 0 || threadIdx.x >= 64) return;
    gw = 0;
    nw = 1;
  } else {
    gw = (int64_t)blockIdx.x * (kSgnsThreads / 64) + wid;
    nw = (int64_t)gridDim.x * (kSgnsThreads / 64);
  }
  const int64_t E = *a.n_examples;
  const int D = a.D;
  const int64_t tbytes = (int64_t)a.V * a.ld * 4;
  const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.rd0, tbytes);
  const __amdgpu_buffer_rsrc_t r1 = make_rsrc(a.rd1, tbytes);
  const __amdgpu_buffer_rsrc_t w0 = make_rsrc(a.wr0, tbytes);
  const __amdgpu_buffer_rsrc_t w1 = make_rsrc(a.wr1, tbytes);
  const int hot = (MODE == kModeSequential || MODE == kModeMinibatch) ? 0 : a.hot_rows;
  const int rowb = (int)a.ld * 4;  // row stride in bytes
  bool on[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) on[v] = (lane + 64 * v) < a.nvec;
  bool eon[NE];
#pragma unroll
  for (int i = 0; i < NE; ++i) eon[i] = (lane + 64 * i) < D;

  for (int64_t c = gw; c * kChunk < E; c += nw) {
    const int64_t e_end = (c * kChunk + kChunk < E) ? c * kChunk + kChunk : E;
    for (int64_t e = c * kChunk; e < e_end; ++e) {
      const int32_t* __restrict__ r = a.rec + e * a.rec_stride;
      int32_t tg[NT];
      tg[0] = r[0];
      const int32_t input = r[1];
      const float alpha = __int_as_float(r[2]);
#pragma unroll
      for (int d = 0; d < K; ++d) tg[d + 1] = r[3 + d];

      // gather: syn0[input] (frozen for the example) and the K+1 syn1neg rows
      float4 l1[NV], rw[NT][NV];
      const int in_off = input * rowb + lane * 16;
#pragma unroll
      for (int v = 0; v < NV; ++v)
        l1[v] = on[v] ? bload4<LA>(r0, in_off + 1024 * v) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        const int off = (tg[d] < 0 ? 0 : tg[d]) * rowb + lane * 16;
#pragma unroll
        for (int v = 0; v < NV; ++v)
          rw[d][v] = (on[v] && tg[d] >= 0) ? bload4<LA>(r1, off + 1024 * v)
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      bool any_hot = false;
#pragma unroll
      for (int d = 0; d < NT; ++d) any_hot |= (tg[d] >= 0 && tg[d] < hot);
      // element layout of syn0[input] for coalesced atomics (hot targets only)
      float l1e[NE];
      if (any_hot) {
#pragma unroll
        for (int i = 0; i < NE; ++i)
          l1e[i] = eon[i] ? bload1<LA>(r0, input * rowb + (lane + 64 * i) * 4) : 0.f;
      }

      // K+1 dots, products exact in fp64, summed in fp64 (dsdot semantics)
      double pd[NT], dot[NT];
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        double s = 0.0;
#pragma unroll
        for (int v = 0; v < NV; ++v) s = dot4(l1[v], rw[d][v], s);
        pd[d] = s;
      }
      wave_reduce_multi<NT>(pd, dot, lane);

      float4 work[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) work[v] = make_float4(0.f, 0.f, 0.f, 0.f);
      bool dirty[NT];
      bool any = false;
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        dirty[d] = false;
        if (tg[d] < 0) continue;
        double dt = dot[d];
        // a repeated target sees its own earlier update (gensim order)
        bool prev_dirty = false;
#pragma unroll
        for (int d2 = 0; d2 < d; ++d2) {
          if (tg[d2] == tg[d]) {
#pragma unroll
            for (int v = 0; v < NV; ++v) rw[d][v] = rw[d2][v];
            prev_dirty = dirty[d2];
          }
        }
        if (prev_dirty) {
          double s = 0.0;
#pragma unroll
          for (int v = 0; v < NV; ++v) s = dot4(l1[v], rw[d][v], s);
          dt = wave_allreduce_d(s);
          dirty[d] = true;
        }
        const float f = (float)dt;
        if (f <= -(float)kMaxExp || f >= (float)kMaxExp) continue;
        const int idx = (int)((f + (float)kMaxExp) * (float)kLutScale);
        const float g = ((d == 0 ? 1.0f : 0.0f) - s_lut[idx]) * alpha;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          work[v].x = __fmaf_rn(g, rw[d][v].x, work[v].x);
          work[v].y = __fmaf_rn(g, rw[d][v].y, work[v].y);
          work[v].z = __fmaf_rn(g, rw[d][v].z, work[v].z);
          work[v].w = __fmaf_rn(g, rw[d][v].w, work[v].w);
          rw[d][v].x = __fmaf_rn(g, l1[v].x, rw[d][v].x);
          rw[d][v].y = __fmaf_rn(g, l1[v].y, rw[d][v].y);
          rw[d][v].z = __fmaf_rn(g, l1[v].z, rw[d][v].z);
          rw[d][v].w = __fmaf_rn(g, l1[v].w, rw[d][v].w);
        }
        if (tg[d] < hot) {
          float* row = a.wr1 + (int64_t)tg[d] * a.ld + lane;
#pragma unroll
          for (int i = 0; i < NE; ++i)
            if (eon[i]) atomicAdd(row + 64 * i, g * l1e[i]);
        }
        dirty[d] = true;
        any = true;
      }

      // write-back: each touched cold syn1neg row once (its last occurrence)
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        bool later = false;
#pragma unroll
        for (int d2 = d + 1; d2 < NT; ++d2) later |= (tg[d2] == tg[d]);
        if (!dirty[d] || later || tg[d] < hot) continue;
        const int off = tg[d] * rowb + lane * 16;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          if (!on[v]) continue;
          if (MODE == kModeMinibatch) {
            const float4 o = bload4<0>(r1, off + 1024 * v);
            float* p = a.wr1 + (int64_t)tg[d] * a.ld + (lane + 64 * v) * 4;
            atomicAdd(p + 0, rw[d][v].x - o.x);
            atomicAdd(p + 1, rw[d][v].y - o.y);
            atomicAdd(p + 2, rw[d][v].z - o.z);
            atomicAdd(p + 3, rw[d][v].w - o.w);
          } else {
            bstore4<SA>(w1, off + 1024 * v, rw[d][v]);
          }
        }
      }
      if (any) {
        const float lf = a.lockf[input];
        if (input < hot) {
          // transpose work to element layout through LDS, then coalesced atomics
          float* sw = s_work[wid];
#pragma unroll
          for (int v = 0; v < NV; ++v)
            *reinterpret_cast<float4*>(sw + (lane + 64 * v) * 4) = work[v];
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
          float* row = a.wr0 + (int64_t)input * a.ld + lane;
#pragma unroll
          for (int i = 0; i < NE; ++i)
            if (eon[i]) atomicAdd(row + 64 * i, lf * sw[lane + 64 * i]);
          __builtin_amdgcn_wave_barrier();
        } else {
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            if (!on[v]) continue;
            float4 o;
            o.x = __fmaf_rn(lf, work[v].x, l1[v].x);
            o.y = __fmaf_rn(lf, work[v].y, l1[v].y);
            o.z = __fmaf_rn(lf, work[v].z, l1[v].z);
            o.w = __fmaf_rn(lf, work[v].w, l1[v].w);
            if (MODE == kModeMinibatch) {
              float* p = a.wr0 + (int64_t)input * a.ld + (lane + 64 * v) * 4;
              atomicAdd(p + 0, o.x - l1[v].x);
              atomicAdd(p + 1, o.y - l1[v].y);
              atomicAdd(p + 2, o.z - l1[v].z);
              atomicAdd(p + 3, o.w - l1[v].w);
            } else {
              bstore4<SA>(w0, in_off + 1024 * v, o);
            }
          }
        }
      }
    }
  }
}


// ---------------------------------------------------------------------------
// k_sgns_atomic: the production Hogwild kernel
// ---------------------------------------------------------------------------
// Same per-example math as k_sgns, but every table update is a memory-side
// float atomic of the delta (g * syn0[input] into syn1neg[t], lockf * work
// into syn0[input]).  With ~4k examples in flight on 256 CUs every row of a
// 24k-gene vocabulary is touched every few microseconds, so plain
// read-modify-write stores lose most updates (measured: iteration-0 loss 4.15
// vs 2.77 sequential); atomics keep all of them (2.76).
//
// Pipelining: example e+1's record and rows are loaded BEFORE example e's
// atomics are issued, so the loads never wait behind the atomics in the
// wave's in-order vmcnt.  l1 and work are staged through LDS in element order
// so each atomic wave-instruction adds 64 contiguous floats (256 B); the
// D % 64 tails of all K+2 rows are packed into shared instructions.
template <int K, int NV>
struct ExRegs {
  int32_t tg[K + 1];
  int32_t input;
  float alpha;
  float4 l1[NV];
  float4 rw[K + 1][NV];
};

// row t of table tbl (0 = syn0, 1 = syn1neg) as this lane's float4 column(s):
// main row plus its stripe copies when t is a striped hot row
template <int NV>
__device__ __forceinline__ void load_row(float4 (&o)[NV], const SgnsArgs& a,
                                         __amdgpu_buffer_rsrc_t rmain, int t, int tbl, int rowb,
                                         int lane, const bool (&on)[NV]) {
  const int off = t * rowb + lane * 16;
#pragma unroll
  for (int v = 0; v < NV; ++v)
    o[v] = on[v] ? bload4<0>(rmain, off + 1024 * v) : make_float4(0.f, 0.f, 0.f, 0.f);
  if (t < a.stripe_rows) {
    const float* sb = a.stripe + (int64_t)tbl * (a.stripe_copies - 1) * a.stripe_rows * a.ld;
    for (int c = 1; c < a.stripe_copies; ++c) {
      const float4* sr = reinterpret_cast<const float4*>(
          sb + ((int64_t)(c - 1) * a.stripe_rows + t) * a.ld);
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        if (!on[v]) continue;
        const float4 q = sr[lane + 64 * v];
        o[v].x += q.x;
        o[v].y += q.y;
        o[v].z += q.z;
        o[v].w += q.w;
      }
    }
  }
}

// destination of an atomic delta for row t of table tbl: main or stripe copy c
__device__ __forceinline__ float* upd_row(const SgnsArgs& a, int tbl, int t, int c) {
  if (c == 0 || t >= a.stripe_rows) return (tbl ? a.wr1 : a.wr0) + (int64_t)t * a.ld;
  return a.stripe + (((int64_t)tbl * (a.stripe_copies - 1) + (c - 1)) * a.stripe_rows + t) * a.ld;
}

template <int K, int NV>
__device__ __forceinline__ void load_example(ExRegs<K, NV>& x, const SgnsArgs& a, int64_t e,
                                             __amdgpu_buffer_rsrc_t r0,
                                             __amdgpu_buffer_rsrc_t r1, int rowb, int lane,
                                             const bool (&on)[NV]) {
  const int32_t* r = a.rec + e * a.rec_stride;
  x.tg[0] = __builtin_amdgcn_readfirstlane(r[0]);
  x.input = __builtin_amdgcn_readfirstlane(r[1]);
  x.alpha = __int_as_float(__builtin_amdgcn_readfirstlane(r[2]));
#pragma unroll
  for (int d = 0; d < K; ++d) x.tg[d + 1] = __builtin_amdgcn_readfirstlane(r[3 + d]);
  load_row<NV>(x.l1, a, r0, x.input, 0, rowb, lane, on);
#pragma unroll
  for (int d = 0; d <= K; ++d) {
    if (x.tg[d] >= 0) {
      load_row<NV>(x.rw[d], a, r1, x.tg[d], 1, rowb, lane, on);
    } else {
#pragma unroll
      for (int v = 0; v < NV; ++v) x.rw[d][v] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// WR (debug ablation only): 0 atomics (production), 1 same-shape plain stores,
// 2 no table writes
template <int WR>
__device__ __forceinline__ void upd(float* p, float v) {
  if (WR == 0) atomicAdd(p, v);
  else if (WR == 1) *p = v;
}

template <int K, int NV, int WR = 0>
__global__ __launch_bounds__(kSgnsThreads) void k_sgns_atomic(SgnsArgs a) {
  constexpr int NT = K + 1;
  constexpr int W = kSgnsThreads / 64;
  __shared__ float s_lut[kExpTableSize];
  __shared__ float s_l1[W][256 * NV];
  __shared__ float s_wk[W][256 * NV];
  for (int i = threadIdx.x; i < kExpTableSize; i += kSgnsThreads) s_lut[i] = a.exp_table[i];
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int64_t gw = (int64_t)blockIdx.x * W + wid;
  const int64_t nw = (int64_t)gridDim.x * W;
  const int64_t E = *a.n_examples;
  const int D = a.D;
  const int full = D >> 6;           // whole 64-float atomic groups per row
  const int tail = D & 63;           // leftover floats per row
  const int tpack = tail ? 64 / tail : 0;  // row tails per packed instruction
  const int64_t tbytes = (int64_t)a.V * a.ld * 4;
  const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.rd0, tbytes);
  const __amdgpu_buffer_rsrc_t r1 = make_rsrc(a.rd1, tbytes);
  const int rowb = (int)a.ld * 4;
  float* s1 = s_l1[wid];
  float* sw = s_wk[wid];
  bool on[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) on[v] = (lane + 64 * v) < a.nvec;

  for (int64_t c = gw; c * kChunk < E; c += nw) {
    const int64_t e_beg = c * kChunk;
    const int64_t e_end = (e_beg + kChunk < E) ? e_beg + kChunk : E;
    ExRegs<K, NV> x;
    load_example<K, NV>(x, a, e_beg, r0, r1, rowb, lane, on);
    for (int64_t e = e_beg; e < e_end; ++e) {
      // ---- compute example e ------------------------------------------------
      double pd[NT], dot[NT];
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        double s = 0.0;
#pragma unroll
        for (int v = 0; v < NV; ++v) s = dot4(x.l1[v], x.rw[d][v], s);
        pd[d] = s;
      }
      wave_reduce_multi<NT>(pd, dot, lane);
      float4 work[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) work[v] = make_float4(0.f, 0.f, 0.f, 0.f);
      float g[NT];
      bool dirty[NT];
      bool any = false;
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        g[d] = 0.f;
        dirty[d] = false;
        if (x.tg[d] < 0) continue;
        double dt = dot[d];
        bool prev_dirty = false;
#pragma unroll
        for (int d2 = 0; d2 < d; ++d2) {
          if (x.tg[d2] == x.tg[d]) {
#pragma unroll
            for (int v = 0; v < NV; ++v) x.rw[d][v] = x.rw[d2][v];
            prev_dirty = dirty[d2];
          }
        }
        if (prev_dirty) {
          double s = 0.0;
#pragma unroll
          for (int v = 0; v < NV; ++v) s = dot4(x.l1[v], x.rw[d][v], s);
          dt = wave_allreduce_d(s);
          dirty[d] = true;
        }
        const float f = (float)dt;
        if (f <= -(float)kMaxExp || f >= (float)kMaxExp) continue;
        const int idx = (int)((f + (float)kMaxExp) * (float)kLutScale);
        const float gg = ((d == 0 ? 1.0f : 0.0f) - s_lut[idx]) * x.alpha;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          work[v].x = __fmaf_rn(gg, x.rw[d][v].x, work[v].x);
          work[v].y = __fmaf_rn(gg, x.rw[d][v].y, work[v].y);
          work[v].z = __fmaf_rn(gg, x.rw[d][v].z, work[v].z);
          work[v].w = __fmaf_rn(gg, x.rw[d][v].w, work[v].w);
          x.rw[d][v].x = __fmaf_rn(gg, x.l1[v].x, x.rw[d][v].x);
          x.rw[d][v].y = __fmaf_rn(gg, x.l1[v].y, x.rw[d][v].y);
          x.rw[d][v].z = __fmaf_rn(gg, x.l1[v].z, x.rw[d][v].z);
          x.rw[d][v].w = __fmaf_rn(gg, x.l1[v].w, x.rw[d][v].w);
        }
        g[d] = gg;
        dirty[d] = true;
        any = true;
      }
      // stage l1 / work in element order
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        *reinterpret_cast<float4*>(s1 + (lane + 64 * v) * 4) = x.l1[v];
        *reinterpret_cast<float4*>(sw + (lane + 64 * v) * 4) = work[v];
      }
      __builtin_amdgcn_wave_barrier();
      int32_t tg[NT];
#pragma unroll
      for (int d = 0; d < NT; ++d) tg[d] = x.tg[d];
      const int32_t input = x.input;
      const float lf = any ? a.lockf[input] : 0.f;

      // ---- prefetch example e+1 (its loads overtake e's atomics) -------------
      if (e + 1 < e_end) load_example<K, NV>(x, a, e + 1, r0, r1, rowb, lane, on);

      // ---- atomics of example e -----------------------------------------------
      const int cbase = (int)(e % (int64_t)a.stripe_copies);
#pragma unroll
      for (int d = 0; d < NT; ++d) {
        if (g[d] == 0.f) continue;
        float* row = upd_row(a, 1, tg[d], (cbase + d) % a.stripe_copies) + lane;
        for (int i = 0; i < full; ++i) upd<WR>(row + 64 * i, g[d] * s1[64 * i + lane]);
      }
      if (any) {
        float* row = upd_row(a, 0, input, (cbase + NT) % a.stripe_copies) + lane;
        for (int i = 0; i < full; ++i) upd<WR>(row + 64 * i, lf * sw[64 * i + lane]);
      }
      if (tail) {
        // rows q = 0..K: syn1neg[tg[q]] += g[q] * l1; q = K+1: syn0[input] += lf * work
        for (int q0 = 0; q0 < NT + 1; q0 += tpack) {
          const int q = q0 + lane / tail;
          const int el = full * 64 + lane % tail;
          float coef = 0.f;
          int row_t = 0;
#pragma unroll
          for (int d = 0; d < NT; ++d) {
            if (q == d) {
              coef = g[d];
              row_t = tg[d] < 0 ? 0 : tg[d];
            }
          }
          const bool from_work = (q == NT);
          if (from_work) {
            coef = any ? lf : 0.f;
            row_t = input;
          }
          if (lane / tail < tpack && q <= NT && coef != 0.f) {
            const float src = from_work ? sw[el] : s1[el];
            float* row = upd_row(a, from_work ? 0 : 1, row_t, (cbase + q) % a.stripe_copies);
            upd<WR>(row + el, coef * src);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// ---------------------------------------------------------------------------
// vocabulary tables on the device ([ext] prepare_vocab / make_cum_table)
// ---------------------------------------------------------------------------
// pow / sample_int in parallel; the two double sums stay sequential (one
// thread) so the rounding sequence is gensim's.
__global__ void k_vocab_pow(const int64_t* __restrict__ counts, int32_t V, double power,
                            double* __restrict__ cpow) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < V) cpow[i] = pow((double)counts[i], power);
}

__global__ void k_vocab_seq(const int64_t* __restrict__ counts, const double* __restrict__ cpow,
                            int32_t V, double sample, uint32_t* __restrict__ cum,
                            uint32_t* __restrict__ sample_int) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  double z = 0.0;
  int64_t total = 0;
  for (int32_t i = 0; i < V; ++i) {
    z += cpow[i];
    total += counts[i];
  }
  double acc = 0.0;
  for (int32_t i = 0; i < V; ++i) {
    acc += cpow[i];
    cum[i] = (uint32_t)rint(acc / z * 2147483647.0);
  }
  double thr;
  if (sample == 0.0) thr = (double)total;
  else if (sample < 1.0) thr = sample * (double)total;
  else thr = (double)(int64_t)(sample * (3.0 + sqrt(5.0)) / 2.0);
  for (int32_t i = 0; i < V; ++i) {
    const double v = (double)counts[i];
    double p = (sqrt(v / thr) + 1.0) * (thr / v);
    if (p >= 1.0) p = 1.0;
    const double si = rint(p * 4294967296.0);
    sample_int[i] = si >= 4294967295.0 ? 0xffffffffu : (uint32_t)si;  // 2**32 == keep always
  }
}

// bkt[b] = bisect_left(cum, b << kBucketShift), b in [0, kBuckets]
__global__ void k_buckets(const uint32_t* __restrict__ cum, int32_t V, int32_t* __restrict__ bkt) {
  const int32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > kBuckets) return;
  const uint64_t x = (uint64_t)b << kBucketShift;
  int32_t lo = 0, hi = V;
  while (hi > lo) {
    const int32_t mid = (lo + hi) >> 1;
    if ((uint64_t)cum[mid] >= x) hi = mid;
    else lo = mid + 1;
  }
  bkt[b] = lo;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
hipError_t launch_job_sample(bool write, const SampleArgs& a, int64_t n_jobs, hipStream_t st) {
  if (n_jobs <= 0) return hipSuccess;
  if (write)
    hipLaunchKernelGGL(k_job_sample<true>, dim3((unsigned)n_jobs), dim3(kSampleThreads), 0, st, a);
  else
    hipLaunchKernelGGL(k_job_sample<false>, dim3((unsigned)n_jobs), dim3(kSampleThreads), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_scan_jobs(const int32_t* nex, int64_t nj, int64_t* off,
                            unsigned long long* examples_total, hipStream_t st) {
  hipLaunchKernelGGL(k_scan_jobs, dim3(1), dim3(1024), 0, st, nex, nj, off, examples_total);
  return hipGetLastError();
}

hipError_t launch_explicit_records(const int32_t* center, const int32_t* input,
                                   const int32_t* negs, int64_t n, int K, float alpha,
                                   int rec_stride, int32_t* rec, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_explicit_records, dim3(blocks), dim3(256), 0, st, center, input, negs, n, K,
                     alpha, rec_stride, rec);
  return hipGetLastError();
}

template <int K, int NV, int POL>
static hipError_t launch_sgns_knp(const SgnsArgs& a, int mode, int grid, hipStream_t st) {
  switch (mode) {
    case kModeSequential:
      hipLaunchKernelGGL((k_sgns<K, NV, kModeSequential, POL>), dim3(1), dim3(kSgnsThreads), 0, st,
                         a);
      break;
    case kModeMinibatch:
      hipLaunchKernelGGL((k_sgns<K, NV, kModeMinibatch, POL>), dim3(grid), dim3(kSgnsThreads), 0,
                         st, a);
      break;
    default:
      hipLaunchKernelGGL((k_sgns<K, NV, kModeHogwild, POL>), dim3(grid), dim3(kSgnsThreads), 0, st,
                         a);
  }
  return hipGetLastError();
}

template <int K, int NV>
static hipError_t launch_sgns_kn(const SgnsArgs& a, int mode, int pol, int grid, hipStream_t st) {
  if (mode == kModeHogwild && a.hot_rows >= a.V) {
    if (a.debug_write == 1 && K == 5 && NV == 1)
      hipLaunchKernelGGL((k_sgns_atomic<K, NV, 1>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
    else if (a.debug_write == 2 && K == 5 && NV == 1)
      hipLaunchKernelGGL((k_sgns_atomic<K, NV, 2>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
    else
      hipLaunchKernelGGL((k_sgns_atomic<K, NV>), dim3(grid), dim3(kSgnsThreads), 0, st, a);
    return hipGetLastError();
  }
  // sequential / minibatch are parity modes: default policy only
  if (mode == kModeSequential || mode == kModeMinibatch || pol == kPolPlain)
    return launch_sgns_knp<K, NV, kPolPlain>(a, mode, grid, st);
  if (pol == kPolWtRd) return launch_sgns_knp<K, NV, kPolWtRd>(a, mode, grid, st);
  return launch_sgns_knp<K, NV, kPolWt>(a, mode, grid, st);
}

template <int K>
static hipError_t launch_sgns_k(const SgnsArgs& a, int nv, int mode, int pol, int grid,
                                hipStream_t st) {
  if (nv == 1) return launch_sgns_kn<K, 1>(a, mode, pol, grid, st);
  return launch_sgns_kn<K, 2>(a, mode, pol, grid, st);
}

bool sgns_supported(int K, int nv) {
  if (nv != 1 && nv != 2) return false;
  switch (K) {
    case 1: case 2: case 3: case 5: case 10: case 15: case 20: return true;
    default: return false;
  }
}

hipError_t launch_sgns(const SgnsArgs& a, int K, int nv, int mode, int pol, int grid,
                       hipStream_t st) {
  switch (K) {
    case 1: return launch_sgns_k<1>(a, nv, mode, pol, grid, st);
    case 2: return launch_sgns_k<2>(a, nv, mode, pol, grid, st);
    case 3: return launch_sgns_k<3>(a, nv, mode, pol, grid, st);
    case 5: return launch_sgns_k<5>(a, nv, mode, pol, grid, st);
    case 10: return launch_sgns_k<10>(a, nv, mode, pol, grid, st);
    case 15: return launch_sgns_k<15>(a, nv, mode, pol, grid, st);
    case 20: return launch_sgns_k<20>(a, nv, mode, pol, grid, st);
    default: return hipErrorInvalidValue;
  }
}

int sgns_blocks_per_cu(int K, int nv) {
  int nb = 0;
  hipError_t e = hipErrorInvalidValue;
#define G2V_OCC(KK, NN)                                                                  \
  if (K == KK && nv == NN)                                                               \
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_sgns_atomic<KK, NN>,           \
                                                     kSgnsThreads, 0);
  G2V_OCC(1, 1) G2V_OCC(2, 1) G2V_OCC(3, 1) G2V_OCC(5, 1) G2V_OCC(10, 1) G2V_OCC(15, 1)
  G2V_OCC(20, 1) G2V_OCC(1, 2) G2V_OCC(2, 2) G2V_OCC(3, 2) G2V_OCC(5, 2) G2V_OCC(10, 2)
  G2V_OCC(15, 2) G2V_OCC(20, 2)
#undef G2V_OCC
  if (e != hipSuccess || nb <= 0) nb = 1;
  return nb;
}


// fold the stripe copies of the hot rows into the main rows, zero the copies
__global__ void k_fold_stripes(float* syn0, float* syn1, float* stripe, int rows, int copies,
                               int64_t ld, int nvec) {
  const int t = blockIdx.x;      // hot row
  const int tbl = blockIdx.y;    // 0 syn0, 1 syn1neg
  const int col = threadIdx.x;   // float4 column
  if (col >= nvec) return;
  float4* m = reinterpret_cast<float4*>((tbl ? syn1 : syn0) + (int64_t)t * ld) + col;
  float4 acc = *m;
  for (int c = 1; c < copies; ++c) {
    float4* p = reinterpret_cast<float4*>(
                    stripe + (((int64_t)tbl * (copies - 1) + (c - 1)) * rows + t) * ld) + col;
    const float4 q = *p;
    acc.x += q.x;
    acc.y += q.y;
    acc.z += q.z;
    acc.w += q.w;
    *p = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  *m = acc;
}

hipError_t launch_fold_stripes(float* syn0, float* syn1, float* stripe, int rows, int copies,
                               int64_t ld, int nvec, hipStream_t st) {
  if (rows <= 0 || copies <= 1) return hipSuccess;
  hipLaunchKernelGGL(k_fold_stripes, dim3(rows, 2), dim3(128), 0, st, syn0, syn1, stripe, rows,
                     copies, ld, nvec);
  return hipGetLastError();
}

hipError_t launch_vocab(const int64_t* counts, double* cpow, int32_t V, double power,
                        double sample, uint32_t* cum, uint32_t* sample_int, int32_t* bkt,
                        hipStream_t st) {
  hipLaunchKernelGGL(k_vocab_pow, dim3((V + 255) / 256), dim3(256), 0, st, counts, V, power, cpow);
  hipLaunchKernelGGL(k_vocab_seq, dim3(1), dim3(64), 0, st, counts, cpow, V, sample, cum,
                     sample_int);
  hipLaunchKernelGGL(k_buckets, dim3((kBuckets + 1 + 255) / 256), dim3(256), 0, st, cum, V, bkt);
  return hipGetLastError();
}

}  // namespace g2v

// ---------------------------------------------------------------------------
// consumer-side: word similarities for the manuscript target function
// (src/evaluation_target_function.py:38,49 -> gensim wv.similarity =
// dot(unitvec(a), unitvec(b)), unitvec = sscal(1/snrm2(v), v) in float32)
// ---------------------------------------------------------------------------
namespace g2v {

// one wave per row: unit[r] = v[r] * (float)(1 / (float)||v[r]||)
__global__ void k_unitvec(const float* __restrict__ v, int64_t V, int D, float* __restrict__ u) {
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= V) return;
  const float* row = v + r * D;
  double s = 0.0;
  for (int k = lane; k < D; k += 64) s = fma((double)row[k], (double)row[k], s);
  s = wave_allreduce_d(s);
  const float len = (float)sqrt(s);
  const float inv = len > 0.f ? (float)(1.0 / (double)len) : 1.f;
  for (int k = lane; k < D; k += 64) u[r * D + k] = row[k] * inv;
}

// one wave per pair: out[i] = (float) dot(u[a[i]], u[b[i]])
__global__ void k_pair_dot(const float* __restrict__ u, int D, const int32_t* __restrict__ a,
                           const int32_t* __restrict__ b, int64_t n, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  const float* x = u + (int64_t)a[i] * D;
  const float* y = u + (int64_t)b[i] * D;
  double s = 0.0;
  for (int k = lane; k < D; k += 64) s = fma((double)x[k], (double)y[k], s);
  s = wave_allreduce_d(s);
  if (lane == 0) out[i] = (float)s;
}

hipError_t launch_cosine_pairs(const float* v, int64_t V, int D, float* u, const int32_t* a,
                               const int32_t* b, int64_t n, float* out, hipStream_t st) {
  hipLaunchKernelGGL(k_unitvec, dim3((unsigned)((V + 3) / 4)), dim3(256), 0, st, v, V, D, u);
  if (n > 0)
    hipLaunchKernelGGL(k_pair_dot, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, u, D, a, b, n,
                       out);
  return hipGetLastError();
}

}  // namespace g2v
