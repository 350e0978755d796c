// g2v_internal.h -- constants and kernel argument blocks shared by the
// kernels (g2v_kernels.hip) and the C-ABI implementation (g2v_api.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace g2v {

// gensim 3.4.0 constants ([ext] word2vec_inner.pyx, base_any2vec.py)
constexpr int kMaxExp = 6;
constexpr int kExpTableSize = 1000;
constexpr int kLutScale = kExpTableSize / kMaxExp / 2;  // C integer division: 83
constexpr int kBatchWords = 10000;                      // batch_words == MAX_SENTENCE_LEN
constexpr uint64_t kLcgMask = 281474976710655ULL;       // 2**48 - 1

// LCG jump tables: n = lo + 2048 * hi, n < 2**22 (draws per job stay far below:
// <= 10000 downsampling draws + K * 20000 negative draws)
constexpr int kJumpBits = 11;
constexpr int kJumpTab = 1 << kJumpBits;
constexpr uint32_t kMaxJump = 1u << (2 * kJumpBits);

// cum_table bucket index: x in [0, 2**31) -> bucket x >> 15 (65536 buckets)
constexpr int kBucketShift = 15;
constexpr int kBuckets = 1 << (31 - kBucketShift);

constexpr int kSampleThreads = 1024;
// k_sgns_atomic addresses the stripe buffer with 32-bit buffer offsets and
// masks unused copies with an offset past it: the buffer stays below 1 GiB
constexpr int64_t kStripeMaxBytes = 1ll << 30;
// stripe buffer layout [table][hot row][copy 1..copies-1][ld]: the copies of
// one row are adjacent (spread over consecutive lines / channels, read as one
// contiguous run); row index of copy c of row t of table tbl
__host__ __device__ inline int64_t stripe_row(int tbl, int t, int c, int rows, int copies) {
  return ((int64_t)tbl * rows + t) * (copies - 1) + (c - 1);
}
constexpr int kSgnsThreads = 256;
constexpr int kChunk = 32;  // consecutive examples a wave trains per grid-stride step

constexpr int kModeHogwild = 0;
constexpr int kModeSequential = 1;
constexpr int kModeMinibatch = 2;

struct LcgJump {
  const uint64_t* a_lo;
  const uint64_t* c_lo;
  const uint64_t* a_hi;
  const uint64_t* c_hi;
};

struct SampleArgs {
  const int32_t* tok;
  const int64_t* sent_off;  // nullptr when sent_len > 0
  int64_t sent_len;
  const int64_t* job_sent;  // [n_jobs+1] (absolute sentence index)
  const uint64_t* job_seed;
  const float* job_alpha;
  int64_t job0;             // first job of this segment
  const uint32_t* sample_int;
  int sample_on;
  const uint32_t* cum;
  const int32_t* bkt;
  int32_t V;
  LcgJump jump;
  int K;
  int rec_stride;           // int32 words per record
  int32_t* job_nex;         // [seg jobs]
  const int64_t* job_exoff; // [seg jobs + 1]
  int32_t* rec;
  unsigned long long* counters;  // [0] effective words, [1] examples, [2] raw words,
                                 // [3] fault bits (kFault*)
};

// sampler fault bits (counters[3]), reported by g2v_sync / g2v_read_stats
constexpr unsigned long long kFaultTokenRange = 1;  // corpus id outside [-1, V)
constexpr unsigned long long kFaultJobSize = 2;     // multi-sentence job > kBatchWords raw words

constexpr int kStampWords = 16;  // g2v_debug_stamps: segment sums, counts, clocks

struct SgnsArgs {
  const int32_t* rec;       // [E][rec_stride]: center, input, alpha bits, negs[K]
  int rec_stride;
  const int64_t* n_examples;  // device scalar E
  const float* rd0;         // syn0 rows read
  const float* rd1;         // syn1neg rows read
  float* wr0;               // syn0 rows written (== rd0 unless MINIBATCH)
  float* wr1;
  const float* lockf;       // [V]
  int64_t ld;               // row stride (floats), multiple of 4
  int nvec;                 // ceil(D / 4): active float4 columns
  int D;
  int V;
  int hot_rows;             // rows [0, hot_rows) are updated with float atomics
  int debug_write;          // 0 production, 2 no table writes (gather roof), 8 stamps;
                            // the -DG2V_ABLATIONS build adds 1, 3, 4, 5, 9
  const float* exp_table;   // [1000]
  // hot-row striping (k_sgns_atomic): rows [0, stripe_rows) of each table have
  // stripe_copies-1 extra copies; value = main + sum(copies), atomics spread
  float* stripe;            // [2][stripe_copies-1][stripe_rows][ld]
  int stripe_rows;
  int stripe_copies;        // 1 = off
  // second tier: rows [stripe_rows, stripe2_rows) with stripe2_copies-1 extra
  // copies each (a power of two), layout [table][row - stripe_rows][copy][ld]
  float* stripe2;
  int stripe2_rows;         // <= stripe_rows = off
  int stripe2_copies;
  int skip_copy_reads;      // ablation build (G2V_OPT_DEBUG_WRITE 6/7): readers ignore copies
  int overlap;              // G2V_OPT_ATOMIC_OVERLAP
  int active_waves;         // G2V_OPT_ACTIVE_WAVES: waves per workgroup that train (1..4)
  unsigned int* queue;      // k_sgns_atomic chunk counter, zeroed before every launch
  uint32_t* dbg16;          // ablation 3 only: packed-f16 scratch, [2][V + stripe rows][ld/2]
  unsigned long long* stamps;  // debug_write 8: per-segment cycle sums (g2v_debug_stamps)
  // stability cap (k_sgns_atomic): waves that train =
  // min(grid x active_waves, cap_budget / (cap_coef x max_r |syn1neg[r]|^2)),
  // the norm read from *norm_bits (float bits) on the device, refreshed before
  // every launch; norm_bits == nullptr: every wave trains
  const unsigned int* norm_bits;
  float cap_coef;           // p_tok_max x (K+1) x the launch's largest alpha
  float cap_budget;
  int* waves_out;           // the waves that trained (block 0 writes it)
  int tail_row0;            // G2V_OPT_TAIL_STORE: syn0 rows >= this and syn1neg
  int tail_row1;            // rows >= tail_row1 take plain stores (k_sgns_atomic)
  // compute_loss ([ext] fast_sentence_sg_neg's LOG_TABLE tally)
  int compute_loss;
  const float* log_table;   // [1000] (float)log(EXP_TABLE[i])
  float* loss_f32;          // sequential: gensim's float32 running sum, continued
  double* loss_f64;         // parallel modes: per-wave float partials summed in double
};

hipError_t launch_job_sample(bool write, const SampleArgs& a, int64_t n_jobs, hipStream_t st);
hipError_t launch_scan_jobs(const int32_t* nex, int64_t nj, int64_t* off,
                            unsigned long long* examples_total, hipStream_t st);
hipError_t launch_explicit_records(const int32_t* center, const int32_t* input,
                                   const int32_t* negs, int64_t n, int K, float alpha,
                                   int rec_stride, int32_t* rec, hipStream_t st);
// negative counts compiled into the SGNS kernels; g2v_sgns.hip and
// g2v_sgns_atomic.hip are built once per K (-DG2V_K=K) and define the per-K
// entry points below; the dispatchers live in g2v_kernels.hip
#define G2V_FOR_EACH_K(X)                                                                  \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)  \
  X(17) X(18) X(19) X(20)
#define G2V_DECL_K(KK)                                                                     \
  hipError_t launch_sgns_k##KK(const SgnsArgs& a, int nv, int mode, int pol, int grid,     \
                               hipStream_t st);                                            \
  hipError_t launch_sgns_atomic_k##KK(const SgnsArgs& a, int nv, int grid, hipStream_t st); \
  int sgns_blocks_per_cu_k##KK(int nv);
G2V_FOR_EACH_K(G2V_DECL_K)
bool sgns_supported(int K, int nv);
hipError_t launch_sgns(const SgnsArgs& a, int K, int nv, int mode, int pol, int grid,
                       hipStream_t st);
hipError_t launch_sgns_atomic(const SgnsArgs& a, int K, int nv, int grid, hipStream_t st);
int sgns_blocks_per_cu(int K, int nv);
hipError_t launch_fold_stripes(float* syn0, float* syn1, float* stripe, int rows, int copies,
                               int64_t ld, int nvec, hipStream_t st);
// replica merge (g2v_average*): rows of one [V][ld] table per call
//   delta:  t <- t - old; cnt[row] = any(t - old != 0); nsq[row] = |t - old|^2
//   apply:  touch: old <- old + t / max(1, max(cnt, 1)^beta / gamma);
//           align: old <- old + t / clamp(|t|^2 / nsq, 1, cnt);
//           mean: old <- t * inv_n;  t <- old
//   local:  the whole merge over n replicas of one device (D <= 512)
constexpr int kMaxLocalReplicas = 16;
struct LocalMergeArgs {
  float* t[kMaxLocalReplicas];
  float* old[kMaxLocalReplicas];
};
hipError_t launch_merge_delta(float* t, const float* old, float* cnt, float* nsq, int64_t V,
                              int64_t ld, int nvec, hipStream_t st);
hipError_t launch_merge_apply(float* t, float* old, const float* cnt, const float* nsq, int64_t V,
                              int64_t ld, int nvec, int rule, float inv_n, float beta, float gamma,
                              hipStream_t st);
hipError_t launch_merge_local(const LocalMergeArgs& a, int n, int64_t V, int64_t ld, int nvec,
                              int rule, float beta, float gamma, hipStream_t st);
// in-process replica group (g2v_comm_init_local): dst = sum over n sources,
// added in source order from 0.f (k_merge_local's order)
struct SumArgs {
  const float* src[kMaxLocalReplicas];
};
hipError_t launch_sum_replicas(const SumArgs& a, int n, float* dst, int64_t count,
                               hipStream_t st);
hipError_t launch_cosine_pairs(const float* v, int64_t V, int D, float* u, const int32_t* a,
                               const int32_t* b, int64_t n, float* out, hipStream_t st);
// Keyed pseudo-random permutation of [0, n) (the device reshuffle of the
// pair corpus, g2v_permute_items8): a 6-round balanced Feistel network on 2h
// bits (4^h >= n) with splitmix64-finalizer round functions, cycle-walked
// into [0, n).  Restated in oracle/shuffle_oracle.py.
struct PermKey {
  uint64_t k[6];
  uint64_t n;
  int half;  // h
};
__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xbf58476d1ce4e5b9ull;
  z ^= z >> 27;
  z *= 0x94d049bb133111ebull;
  z ^= z >> 31;
  return z;
}
inline PermKey perm_key(uint64_t n, uint64_t seed) {
  PermKey pk{};
  pk.n = n;
  pk.half = 1;
  while (pk.half < 31 && (1ull << (2 * pk.half)) < n) ++pk.half;
  for (int r = 0; r < 6; ++r) pk.k[r] = mix64(seed + 0x9e3779b97f4a7c15ull * (uint64_t)(r + 1));
  return pk;
}
__host__ __device__ inline uint64_t perm_at(const PermKey& pk, uint64_t i) {
  const uint64_t mask = (1ull << pk.half) - 1;
  uint64_t y = i;
  do {
    uint64_t L = y >> pk.half, R = y & mask;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const uint64_t t = L ^ (mix64(R ^ pk.k[r]) & mask);
      L = R;
      R = t;
    }
    y = (L << pk.half) | R;
  } while (y >= pk.n);
  return y;
}
hipError_t launch_permute8(const uint64_t* src, uint64_t* dst, const PermKey& pk, int64_t first,
                           int64_t count, hipStream_t st);
hipError_t launch_first_occ_perm8(const uint64_t* src, const PermKey& pk, int32_t n_ids,
                                  int64_t* first, hipStream_t st);
hipError_t launch_vocab(const int64_t* counts, double* cpow, int32_t V, double power,
                        double sample, uint32_t* cum, uint32_t* sample_int, int32_t* bkt,
                        hipStream_t st);

// record an error for g2v_last_error() (g2v_api.hip); returns code
int set_error(int code, const std::string& msg);

// host side: LCG jump tables (g2v_host.cpp)
void lcg_jump_tables(uint64_t* a_lo, uint64_t* c_lo, uint64_t* a_hi, uint64_t* c_hi);

}  // namespace g2v
