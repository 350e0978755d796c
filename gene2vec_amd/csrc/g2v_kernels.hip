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
//   k_sgns* (g2v_sgns.hip, g2v_sgns_atomic.hip)
//                        the update: ONE WAVE PER DIRECTED EXAMPLE, lane l owns
//                        float4 columns l (+64): 16-B row gathers from
//                        syn0/syn1neg, K+1 dots in fp64 (dsdot) reduced across the
//                        wave by a value-halving xor butterfly, LUT sigmoid from
//                        LDS, gradient + work accumulation in registers, and
//                        plain (Hogwild) float4 write-back of every touched row.
//
// Everything is memory-gather bound (0.68 flop/B): no MFMA by design.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>

#include "g2v_device.h"

namespace g2v {

// ---------------------------------------------------------------------------
// k_job_sample: one workgroup per job ([ext] train_batch_sg pre-pass)
// ---------------------------------------------------------------------------
//
// gensim's train_batch_sg stops collecting at MAX_SENTENCE_LEN = 10000
// effective words (the token that makes the 10000th kept word is the last one
// that draws).  g2v_plan_jobs gives a sentence longer than batch_words a job of
// its own, so a job of n > kBatchWords raw words is one sentence: its kept
// prefix is collected chunk by chunk and the scan stops at the cut.
template <bool WRITE>
__global__ __launch_bounds__(kSampleThreads) void k_job_sample(SampleArgs a) {
  __shared__ int32_t s_eff[kBatchWords];       // kept tokens, compacted
  __shared__ uint16_t s_kc[kBatchWords];       // kept-before count per raw position
  __shared__ int s_scan[kSampleThreads / 64];
  __shared__ long long s_cut_draws;            // draws up to the 10000th kept word, -1 = no cut
  __shared__ int s_bad;

  const int64_t j = blockIdx.x;                // job within segment
  const int64_t jg = a.job0 + j;
  const int64_t s0 = a.job_sent[jg], s1 = a.job_sent[jg + 1];
  const int64_t tb = sent_start(a, s0);
  const int64_t n_raw = sent_start(a, s1) - tb;
  const int ns_raw = (int)(s1 - s0);
  // more than kBatchWords raw words in several sentences cannot come from
  // g2v_plan_jobs (a host CSR is checked; a device CSR is not): train nothing
  const bool bad_job = n_raw > kBatchWords && ns_raw > 1;
  const int64_t n = bad_job ? 0 : n_raw;
  const int ns = bad_job ? 0 : ns_raw;
  const uint64_t seed = a.job_seed[jg];
  if (threadIdx.x == 0) {
    s_cut_draws = -1;
    s_bad = 0;
  }
  __syncthreads();

  int64_t inv_base = 0;
  int keep_base = 0;
  for (int64_t t0 = 0; t0 < n && keep_base < kBatchWords; t0 += kSampleThreads) {
    const int64_t t = t0 + threadIdx.x;
    int32_t w = (t < n) ? a.tok[tb + t] : -1;
    if (w < -1 || w >= a.V) {  // not a vocabulary index: skipped like OOV, reported
      s_bad = 1;
      w = -1;
    }
    const int inv = (w >= 0);
    int tot_inv;
    const int64_t p = inv_base + block_excl_scan<kSampleThreads>(inv, s_scan, tot_inv);
    int keep = inv;
    if (inv && a.sample_on) {
      // gensim: drop iff sample_int < random_int32(&next_random); the p-th draw
      const uint32_t r = (uint32_t)(lcg_jump_big(seed, (uint64_t)p, a.jump) >> 16);
      keep = !(a.sample_int[w] < r);
    }
    int tot_keep;
    const int c = keep_base + block_excl_scan<kSampleThreads>(keep, s_scan, tot_keep);
    if (t < kBatchWords) s_kc[t] = (uint16_t)(c < kBatchWords ? c : kBatchWords);
    if (keep && c < kBatchWords) s_eff[c] = w;
    if (keep && c == kBatchWords - 1) s_cut_draws = p + 1;
    inv_base += tot_inv;
    keep_base += tot_keep;
  }
  __syncthreads();
  const int kept = keep_base < kBatchWords ? keep_base : kBatchWords;

  const uint64_t ndraw =
      a.sample_on ? (s_cut_draws >= 0 ? (uint64_t)s_cut_draws : (uint64_t)inv_base) : 0ull;
  const float alpha = WRITE ? a.job_alpha[jg] : 0.f;
  const int64_t out_base = WRITE ? a.job_exoff[j] : 0;
  const uint32_t cum_last = a.cum[a.V - 1];
  int ex_base = 0;
  for (int q0 = 0; q0 < ns; q0 += kSampleThreads) {
    const int q = q0 + threadIdx.x;
    int e0 = 0, e1 = 0;
    if (q < ns) {
      // kept-before count at a sentence boundary (the job end: all kept words)
      const int64_t b0 = sent_start(a, s0 + q) - tb, b1 = sent_start(a, s0 + q + 1) - tb;
      e0 = b0 >= n ? kept : s_kc[b0];
      e1 = b1 >= n ? kept : s_kc[b1];
    }
    const int L = e1 - e0;
    const int nex = L >= 2 ? 2 * (L - 1) : 0;  // window 1: (i,i-1),(i,i+1) in range
    int tot;
    const int eb = ex_base + block_excl_scan<kSampleThreads>(nex, s_scan, tot);
    // example k of a sentence of L kept words, in gensim's loop order:
    // k = 0 -> (0, 1); k >= 1 -> i = (k+1)/2, j = i-1 (k odd) or i+1 (k even)
    auto write_rec = [&](int e, int i, int jj) {
      int32_t* r = a.rec + (out_base + e) * a.rec_stride;
      const int32_t center = s_eff[i];
      r[0] = center;
      r[1] = s_eff[jj];
      r[2] = __float_as_int(alpha);
      uint64_t nr = lcg_jump_big(seed, ndraw + (uint64_t)a.K * (uint64_t)e, a.jump);
      for (int d = 0; d < a.K; ++d) {
        const int32_t t = draw_negative(nr, a.cum, a.bkt, a.V, cum_last);
        r[3 + d] = (t == center) ? -1 : t;
      }
    };
    if (WRITE && ns == 1) {
      // one sentence (long ones always are; it starts at kept word 0): its
      // examples spread over the whole block (tot = its example count)
      for (int k = threadIdx.x; k < tot; k += kSampleThreads) {
        const int i = (k + 1) >> 1;
        const int jj = k == 0 ? 1 : ((k & 1) ? i - 1 : i + 1);
        write_rec(k, i, jj);
      }
    } else if (WRITE && nex) {
      int e = eb;
      for (int i = e0; i < e1; ++i) {
#pragma unroll
        for (int dj = -1; dj <= 1; dj += 2) {
          const int jj = i + dj;
          if (jj < e0 || jj >= e1) continue;
          write_rec(e, i, jj);
          ++e;
        }
      }
    }
    ex_base += tot;
  }
  if (!WRITE && threadIdx.x == 0) {
    a.job_nex[j] = ex_base;
    atomicAdd(a.counters + 0, (unsigned long long)kept);   // effective words
    atomicAdd(a.counters + 2, (unsigned long long)n_raw);  // raw words
    const unsigned long long f = (s_bad ? kFaultTokenRange : 0ull) | (bad_job ? kFaultJobSize : 0ull);
    if (f) atomicOr(a.counters + 3, f);
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


// ---------------------------------------------------------------------------
// SGNS dispatch over the compiled negative counts (one object per K)
// ---------------------------------------------------------------------------
bool sgns_supported(int K, int nv) {
  if (nv != 1 && nv != 2) return false;
  switch (K) {
#define G2V_CASE(KK) case KK:
    G2V_FOR_EACH_K(G2V_CASE)
#undef G2V_CASE
    return true;
    default: return false;
  }
}

hipError_t launch_sgns(const SgnsArgs& a, int K, int nv, int mode, int pol, int grid,
                       hipStream_t st) {
  switch (K) {
#define G2V_CASE(KK) case KK: return launch_sgns_k##KK(a, nv, mode, pol, grid, st);
    G2V_FOR_EACH_K(G2V_CASE)
#undef G2V_CASE
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_sgns_atomic(const SgnsArgs& a, int K, int nv, int grid, hipStream_t st) {
  switch (K) {
#define G2V_CASE(KK) case KK: return launch_sgns_atomic_k##KK(a, nv, grid, st);
    G2V_FOR_EACH_K(G2V_CASE)
#undef G2V_CASE
    default: return hipErrorInvalidValue;
  }
}

int sgns_blocks_per_cu(int K, int nv) {
  switch (K) {
#define G2V_CASE(KK) case KK: return sgns_blocks_per_cu_k##KK(nv);
    G2V_FOR_EACH_K(G2V_CASE)
#undef G2V_CASE
    default: return 1;
  }
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
                    stripe + stripe_row(tbl, t, c, rows, copies) * ld) + col;
    const float4 q = *p;
    acc.x += q.x;
    acc.y += q.y;
    acc.z += q.z;
    acc.w += q.w;
    *p = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  *m = acc;
}

// largest squared row norm of a [V][ld] table (the Hogwild stability cap of
// g2v_train): waves stride over the rows keeping a running maximum, the
// workgroup's maximum goes out as one atomicMax on the float bits (a
// non-negative float orders like its unsigned bits) -- 256 atomics on one word,
// not one per row
constexpr int kNormBlocks = 256;
__global__ void k_row_norm2_max(const float* t, int V, int64_t ld, int D, unsigned int* out) {
  __shared__ float s_max[4];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t waves = (int64_t)gridDim.x * 4;
  float m = 0.f;
  for (int64_t r = (int64_t)blockIdx.x * 4 + w; r < V; r += waves) {
    const float* row = t + r * ld;
    float s = 0.f;
    for (int i = lane; i < D; i += 64) s = fmaf(row[i], row[i], s);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    m = fmaxf(m, s);
  }
  if (lane == 0) s_max[w] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(out, __float_as_uint(fmaxf(fmaxf(s_max[0], s_max[1]), fmaxf(s_max[2], s_max[3]))));
}

hipError_t launch_row_norm2_max(const float* t, int V, int64_t ld, int D, unsigned int* out,
                                hipStream_t st) {
  if (V <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>(kNormBlocks, ((int64_t)V + 3) / 4);
  hipLaunchKernelGGL(k_row_norm2_max, dim3((unsigned)blocks), dim3(256), 0, st, t, V, ld, D, out);
  return hipGetLastError();
}

hipError_t launch_fold_stripes(float* syn0, float* syn1, float* stripe, int rows, int copies,
                               int64_t ld, int nvec, hipStream_t st) {
  if (rows <= 0 || copies <= 1) return hipSuccess;
  hipLaunchKernelGGL(k_fold_stripes, dim3(rows, 2), dim3(128), 0, st, syn0, syn1, stripe, rows,
                     copies, ld, nvec);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// replica merge (g2v_average / g2v_average_local): one wave per row, lane l
// owns float4 columns l, l+64; HBM-bound streaming (rows are 128-B aligned)
// ---------------------------------------------------------------------------
// every lane gets the wave's total (a fixed xor butterfly: the same bits on
// every path that merges, so g2v_average_local and the all-reduce agree)
__device__ __forceinline__ float wave_sum_f(float x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m);
  return x;
}

__device__ __forceinline__ float sq4(float4 d) { return d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w; }

// t <- t - old (the replica's change since the last merge, summed over ranks
// by the all-reduce that follows), cnt[row] = 1 if the row changed, nsq[row] =
// |t - old|^2 (the align rule's denominator once summed over ranks)
__global__ __launch_bounds__(256) void k_merge_delta(float* __restrict__ t,
                                                     const float* __restrict__ old,
                                                     float* __restrict__ cnt,
                                                     float* __restrict__ nsq, int64_t V,
                                                     int64_t ld, int nvec) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= V) return;
  float4* tr = reinterpret_cast<float4*>(t + r * ld);
  const float4* orw = reinterpret_cast<const float4*>(old + r * ld);
  int nz = 0;
  float q = 0.f;
  for (int c = lane; c < nvec; c += 64) {
    const float4 x = tr[c], o = orw[c];
    const float4 d = make_float4(x.x - o.x, x.y - o.y, x.z - o.z, x.w - o.w);
    nz |= (d.x != 0.f) | (d.y != 0.f) | (d.z != 0.f) | (d.w != 0.f);
    q += sq4(d);
    tr[c] = d;
  }
  const int any = __any(nz);
  q = wave_sum_f(q);
  if (lane == 0) {
    cnt[r] = any ? 1.f : 0.f;
    nsq[r] = q;
  }
}

// divisor of the summed change of a row k replicas changed:
//   touch (rule 0): max(1, k^beta / gamma) (beta = gamma = 1: the mean; gamma
//     scales the mean up, bounded by the sum; a row every replica drove to the
//     same point moves gamma times that far)
//   align (rule 2): |sum d|^2 / sum |d|^2 clamped to [1, k] -- k when the
//     replicas' changes agree (a row they all drove to the same point: their
//     mean), 1 when they are orthogonal (independent updates that one model
//     would have applied all of: their sum) -- then shaped by beta / gamma
//     like the touch divisor
__device__ __forceinline__ float touch_div(float k, float beta, float gamma) {
  const float kb = beta == 1.f ? k : powf(k, beta);
  return gamma == 1.f ? kb : fmaxf(1.f, kb / gamma);
}
__device__ __forceinline__ float align_div(float k, float tsq, float nsq) {
  return nsq > 0.f ? fminf(fmaxf(tsq / nsq, 1.f), fmaxf(k, 1.f)) : 1.f;
}

// after the all-reduce: touch / align: t holds sum_r d_r, cnt the number of
// replicas that changed the row, nsq sum_r |d_r|^2: new = old + t / divisor;
// mean (rule 1): t holds sum_r t_r: new = t * inv_n.  All: old = t = new.
__global__ __launch_bounds__(256) void k_merge_apply(float* __restrict__ t, float* __restrict__ old,
                                                     const float* __restrict__ cnt,
                                                     const float* __restrict__ nsq, int64_t V,
                                                     int64_t ld, int nvec, int rule, float inv_n,
                                                     float beta, float gamma) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= V) return;
  float4* tr = reinterpret_cast<float4*>(t + r * ld);
  float4* orw = reinterpret_cast<float4*>(old + r * ld);
  float k = 1.f;
  if (rule == 0) {
    k = touch_div(fmaxf(cnt[r], 1.f), beta, gamma);
  } else if (rule == 2) {
    float q = 0.f;
    for (int c = lane; c < nvec; c += 64) q += sq4(tr[c]);
    k = touch_div(align_div(cnt[r], wave_sum_f(q), nsq[r]), beta, gamma);
  }
  for (int c = lane; c < nvec; c += 64) {
    const float4 x = tr[c];
    float4 nv;
    if (rule != 1) {
      const float4 o = orw[c];
      nv = make_float4(o.x + x.x / k, o.y + x.y / k, o.z + x.z / k, o.w + x.w / k);
    } else {
      nv = make_float4(x.x * inv_n, x.y * inv_n, x.z * inv_n, x.w * inv_n);
    }
    tr[c] = nv;
    orw[c] = nv;
  }
}

// n replicas on one device: the whole merge in one pass (deltas, counts and
// squared norms summed in replica order, as the all-reduce path sums them);
// a lane holds at most 2 float4 columns (D <= 512)
__global__ __launch_bounds__(256) void k_merge_local(LocalMergeArgs a, int n, int64_t V,
                                                     int64_t ld, int nvec, int rule, float beta,
                                                     float gamma) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= V) return;
  const int64_t base = r * ld;
  float kc = 0.f, nq = 0.f;
  float4 s[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
  for (int i = 0; i < n; ++i) {
    const float4* tr = reinterpret_cast<const float4*>(a.t[i] + base);
    const float4* orw = reinterpret_cast<const float4*>(a.old[i] + base);
    int nz = 0;
    float q = 0.f;
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int c = lane + 64 * v;
      if (c >= nvec) continue;
      const float4 x = tr[c];
      if (rule != 1) {
        const float4 o = orw[c];
        const float4 d = make_float4(x.x - o.x, x.y - o.y, x.z - o.z, x.w - o.w);
        nz |= (d.x != 0.f) | (d.y != 0.f) | (d.z != 0.f) | (d.w != 0.f);
        q += sq4(d);
        s[v].x += d.x;
        s[v].y += d.y;
        s[v].z += d.z;
        s[v].w += d.w;
      } else {
        s[v].x += x.x;
        s[v].y += x.y;
        s[v].z += x.z;
        s[v].w += x.w;
      }
    }
    if (rule != 1) {
      kc += __any(nz) ? 1.f : 0.f;
      nq += wave_sum_f(q);
    }
  }
  float kf = 1.f;
  if (rule == 0) {
    kf = touch_div(fmaxf(kc, 1.f), beta, gamma);
  } else if (rule == 2) {
    float q = 0.f;
#pragma unroll
    for (int v = 0; v < 2; ++v)
      if (lane + 64 * v < nvec) q += sq4(s[v]);
    kf = touch_div(align_div(kc, wave_sum_f(q), nq), beta, gamma);
  }
  const float inv_n = 1.f / (float)n;
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int c = lane + 64 * v;
    if (c >= nvec) continue;
    float4 nv;
    if (rule != 1) {
      const float4 o = reinterpret_cast<const float4*>(a.old[0] + base)[c];
      nv = make_float4(o.x + s[v].x / kf, o.y + s[v].y / kf, o.z + s[v].z / kf,
                       o.w + s[v].w / kf);
    } else {
      nv = make_float4(s[v].x * inv_n, s[v].y * inv_n, s[v].z * inv_n, s[v].w * inv_n);
    }
    for (int i = 0; i < n; ++i) {
      reinterpret_cast<float4*>(a.t[i] + base)[c] = nv;
      reinterpret_cast<float4*>(a.old[i] + base)[c] = nv;
    }
  }
}

// the in-process transport's all-reduce (g2v_comm_init_local): dst = sum of n
// replicas' buffers, added in rank order from 0.f -- the order k_merge_local
// sums its deltas in, so a merge over the group equals g2v_average_local's bit
// for bit.  HBM-bound streaming, float4 when every pointer allows it.
template <bool VEC>
__global__ __launch_bounds__(256) void k_sum_replicas(SumArgs a, int n, float* __restrict__ dst,
                                                      int64_t count) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (VEC) {
    const int64_t n4 = count >> 2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int q = 0; q < n; ++q) {
        const float4 x = reinterpret_cast<const float4*>(a.src[q])[i];
        s.x += x.x;
        s.y += x.y;
        s.z += x.z;
        s.w += x.w;
      }
      reinterpret_cast<float4*>(dst)[i] = s;
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
      float s = 0.f;
      for (int q = 0; q < n; ++q) s += a.src[q][i];
      dst[i] = s;
    }
  }
}

hipError_t launch_sum_replicas(const SumArgs& a, int n, float* dst, int64_t count,
                               hipStream_t st) {
  if (count <= 0 || n <= 0) return hipSuccess;
  bool vec = count % 4 == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0;
  for (int q = 0; q < n; ++q) vec = vec && (reinterpret_cast<uintptr_t>(a.src[q]) & 15) == 0;
  const int64_t items = vec ? count / 4 : count;
  const unsigned grid = (unsigned)std::min<int64_t>((items + 255) / 256, 4096);
  if (vec)
    hipLaunchKernelGGL(k_sum_replicas<true>, dim3(grid), dim3(256), 0, st, a, n, dst, count);
  else
    hipLaunchKernelGGL(k_sum_replicas<false>, dim3(grid), dim3(256), 0, st, a, n, dst, count);
  return hipGetLastError();
}

hipError_t launch_merge_delta(float* t, const float* old, float* cnt, float* nsq, int64_t V,
                              int64_t ld, int nvec, hipStream_t st) {
  if (V <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_merge_delta, dim3((unsigned)((V + 3) / 4)), dim3(256), 0, st, t, old, cnt,
                     nsq, V, ld, nvec);
  return hipGetLastError();
}

hipError_t launch_merge_apply(float* t, float* old, const float* cnt, const float* nsq, int64_t V,
                              int64_t ld, int nvec, int rule, float inv_n, float beta, float gamma,
                              hipStream_t st) {
  if (V <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_merge_apply, dim3((unsigned)((V + 3) / 4)), dim3(256), 0, st, t, old, cnt,
                     nsq, V, ld, nvec, rule, inv_n, beta, gamma);
  return hipGetLastError();
}

hipError_t launch_merge_local(const LocalMergeArgs& a, int n, int64_t V, int64_t ld, int nvec,
                              int rule, float beta, float gamma, hipStream_t st) {
  if (V <= 0 || n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_merge_local, dim3((unsigned)((V + 3) / 4)), dim3(256), 0, st, a, n, V, ld,
                     nvec, rule, beta, gamma);
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

// dst[i] = src[perm(first + i)], 8-byte items (an int32 gene pair): the
// per-iteration reshuffle of a device-resident pair corpus, each rank
// gathering only its own shard of the permuted order
__global__ void k_permute8(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst, PermKey pk,
                           int64_t first, int64_t count) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride)
    dst[i] = src[perm_at(pk, (uint64_t)(first + i))];
}

hipError_t launch_permute8(const uint64_t* src, uint64_t* dst, const PermKey& pk, int64_t first,
                           int64_t count, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((count + 255) / 256, 16384);
  hipLaunchKernelGGL(k_permute8, dim3((unsigned)blocks), dim3(256), 0, st, src, dst, pk, first,
                     count);
  return hipGetLastError();
}

// First occurrence of every id in the PERMUTED token stream (position 2i /
// 2i+1 for the two genes of the pair at permuted index i): the vocabulary
// scan of [ext] scan_vocab after a device shuffle -- gensim breaks count ties
// by first occurrence.  A small grid sweeps the order front to back, so the
// frequent ids are set within the first sweep and later threads find a
// smaller value and skip the atomic.
__global__ void k_first_occ_perm8(const uint64_t* __restrict__ src, PermKey pk, int32_t n_ids,
                                  unsigned long long* __restrict__ first) {
  const int64_t n = (int64_t)pk.n;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t item = src[perm_at(pk, (uint64_t)i)];
    const int32_t ab[2] = {(int32_t)(uint32_t)item, (int32_t)(uint32_t)(item >> 32)};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int32_t w = ab[k];
      const unsigned long long pos = 2ull * (unsigned long long)i + (unsigned long long)k;
      if (w >= 0 && w < n_ids && __hip_atomic_load(first + w, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT) > pos)
        atomicMin(first + w, pos);
    }
  }
}

// first[] starts all-ones: an id that never occurs reads -1 as int64
hipError_t launch_first_occ_perm8(const uint64_t* src, const PermKey& pk, int32_t n_ids,
                                  int64_t* first, hipStream_t st) {
  hipError_t e = hipMemsetAsync(first, 0xFF, sizeof(int64_t) * (size_t)n_ids, st);
  if (e != hipSuccess || pk.n == 0) return e;
  const int64_t blocks = std::min<int64_t>(((int64_t)pk.n + 255) / 256, 2048);
  hipLaunchKernelGGL(k_first_occ_perm8, dim3((unsigned)blocks), dim3(256), 0, st, src, pk, n_ids,
                     reinterpret_cast<unsigned long long*>(first));
  return hipGetLastError();
}

}  // namespace g2v
