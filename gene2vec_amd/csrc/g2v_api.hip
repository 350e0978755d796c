// g2v_api.hip -- C ABI of libg2v.so (declared in include/g2v.h).
//
// Owns the device state that gensim keeps in the Word2Vec model object
// ([ext] wv.vectors, trainables.syn1neg, trainables.vectors_lockf,
// vocabulary.cum_table, per-word sample_int) and replaces the per-job hook
// train_batch_sg that gensim's worker threads call (src/gene2vec.py:70,87).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: RCCL is dlopen()ed by g2v_comm_*
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <new>
#include <thread>
#include <string>
#include <utility>
#include <vector>

#include "g2v.h"
#include "g2v_internal.h"

using namespace g2v;

namespace g2v {
hipError_t launch_row_norm2_max(const float* t, int V, int64_t ld, int D, unsigned int* out,
                                hipStream_t st);  // g2v_kernels.hip
}

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess)                                                                  \
      return fail(G2V_EHIP, "%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, \
                  __LINE__);                                                               \
  } while (0)

#define REQUIRE(cond, code, ...)                \
  do {                                                \
    if (!(cond)) return fail((code), __VA_ARGS__);    \
  } while (0)

template <typename T>
int dev_alloc(T** p, size_t n) {
  *p = nullptr;
  if (n == 0) n = 1;
  hipError_t e = hipMalloc((void**)p, n * sizeof(T));
  if (e != hipSuccess)
    return fail(G2V_ENOMEM, "hipMalloc(%zu bytes) failed: %s", n * sizeof(T), hipGetErrorString(e));
  return G2V_OK;
}

template <typename T>
void dev_free(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

// grow a device buffer (contents discarded); caller guarantees no in-flight use
// (stream-ordered: we synchronise the stream before freeing)
template <typename T>
int dev_reserve(hipStream_t st, T** p, int64_t* cap, int64_t need) {
  if (need <= *cap && *p) return G2V_OK;
  if (*p) {
    HIPCHK(hipStreamSynchronize(st));
    dev_free(*p);
  }
  int64_t n = std::max<int64_t>(need, *cap + *cap / 2);
  int rc = dev_alloc(p, (size_t)n);
  if (rc) {
    *cap = 0;
    return rc;
  }
  *cap = n;
  return G2V_OK;
}

}  // namespace

int g2v::set_error(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

enum { kCommNone = 0, kCommRccl = 1, kCommLocal = 2, kCommHost = 3 };

// In-process replica group (g2v_comm_init_local): n contexts of one process on
// one device, each driven by its own host thread, merge through a device sum
// instead of ncclAllReduce -- the RCCL path's delta/apply kernels and in-call
// merges with several replicas on a one-GPU box, where RCCL refuses two ranks
// ("Duplicate GPU detected").  Collectives meet at a host barrier; the data
// dependencies between the ranks' streams are HIP events.
struct g2v_local_group {
  int n = 0;
  int device = -1;
  int32_t V = 0;
  int64_t ld = 0;
  int timeout_s = 600;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::string why;
  std::vector<int> joined;
  std::vector<hipEvent_t> ev;                 // per rank: its buffers are ready
  hipEvent_t ev_done = nullptr;               // rank 0: the sum is in scratch
  std::vector<std::array<float*, 3>> bufs;    // per rank: the buffers of this collective
  float* scratch = nullptr;
  size_t scratch_cap = 0;                     // floats
};

struct g2v_ctx {
  int device = 0;
  int32_t V = 0, D = 0, K = 0, window = 1;
  int nv = 1, nvec = 0, rec_stride = 0;
  int64_t ld = 0;
  int cus = 0, sgns_grid = 0;
  bool grid_user = false;       // G2V_OPT_GRID set explicitly
  double u_max = 0.0;           // hottest row's updates per example (set_vocab)
  double p_tok_max = 0.0;       // hottest row's share of the kept tokens (syn0 input rate)
  int hot_rows = -1;            // -1: default (all rows atomic-updated); tuned via g2v_set_option
  int cache_policy = 1;         // kPolWt
  int debug_write = 0;
  // 4 hottest rows striped (round 5, interleaved A/B against 8 with the 16-copy
  // default: sample 0 +1.5-2.6 %, C4 +1.8 %, C2 +0.1-0.5 %, a 3,000-gene corpus
  // within its noise; 2 rows lose 10 % at sample 0)
  int stripe_rows = 4, stripe_copies = 0;  // copies 0 = auto (stripe_copies_eff)
  int stripe2_rows = -1, stripe2_copies = 4;  // second tier: rows [stripe_rows, stripe2_rows), -1 = auto
  float* stripe2 = nullptr;
  int64_t stripe2_cap = 0;
  int atomic_overlap = 1;
  int tail_store = -1;  // G2V_OPT_TAIL_STORE: -1 auto (collision budget), 0 off, n rows >= n
  // per row (index order) from set_vocab: the suffix max over rows >= r of
  // u(r') = K p_neg(r') + p_tok(r') (syn1neg updates per example), the tail
  // stores' collision budget; non-increasing whatever the count order or
  // ns_exponent, so the auto boundary is a partition point
  std::vector<double> u_row;
  int sample_overlap = 1;  // measured +1.2 % at C2
  int64_t merge_every = 0;  // G2V_OPT_MERGE_EVERY_JOBS: replica merges inside g2v_train
  int64_t debug_fail_merge = 0;  // G2V_OPT_DEBUG_FAIL_MERGE: fault injection
  int merge_rule = 0;
  float merge_beta = 1.0f;   // G2V_OPT_MERGE_BETA_MILLI / 1000
  float merge_gamma = 1.0f;  // G2V_OPT_MERGE_GAMMA_MILLI / 1000
  float* stripe = nullptr;
  int64_t stripe_cap = 0;
  uint32_t* dbg16 = nullptr;  // ablation 3: packed-f16 atomic scratch [2][V + stripes][ld/2]
  int64_t dbg16_cap = 0;
  hipStream_t own_stream = nullptr, stream = nullptr;

  float *own0 = nullptr, *own1 = nullptr;  // context-owned tables
  float *syn0 = nullptr, *syn1 = nullptr;  // active tables (owned or borrowed)
  float* lockf = nullptr;
  float* exp_table = nullptr;
  uint64_t* jump = nullptr;  // 4 x kJumpTab
  uint32_t *cum = nullptr, *sample_int = nullptr;
  int32_t* bkt = nullptr;
  int64_t* d_counts = nullptr;
  double* d_cpow = nullptr;
  int sample_on = 0;
  bool vocab_ready = false, weights_ready = false;

  // corpus
  const int32_t* tok = nullptr;
  const int64_t* sent_off = nullptr;
  int32_t* own_tok = nullptr;
  int64_t* own_off = nullptr;
  int64_t n_tok = 0, n_sent = 0, sent_len = 0;
  std::vector<int64_t> h_sent_off;  // host copy (host-provided CSR only)
  bool corpus_ready = false;

  // job tables
  int64_t job_cap = 0;
  int64_t* d_job_sent = nullptr;
  float* d_job_alpha = nullptr;
  uint64_t* d_job_seed = nullptr;
  int64_t job_alpha_cap = 0, job_seed_cap = 0;
  void* h_stage = nullptr;
  size_t h_stage_cap = 0;
  hipEvent_t stage_ev = nullptr;
  bool stage_pending = false;

  // per-segment workspace
  int64_t seg_jobs = 1024;
  int64_t nex_cap = 0, exoff_cap = 0, rec_cap = 0;
  int32_t* d_job_nex = nullptr;
  int64_t* d_job_exoff = nullptr;
  int32_t* d_rec = nullptr;
  // G2V_OPT_SAMPLE_OVERLAP: a second workspace and a side stream, so segment
  // s+1 is sampled while segment s trains
  int64_t nex_cap2 = 0, exoff_cap2 = 0, rec_cap2 = 0;
  int32_t* d_job_nex2 = nullptr;
  int64_t* d_job_exoff2 = nullptr;
  int32_t* d_rec2 = nullptr;
  hipStream_t side = nullptr;
  hipEvent_t ev_up = nullptr, ev_samp[2] = {nullptr, nullptr}, ev_sgns[2] = {nullptr, nullptr};

  // explicit-step scratch
  int64_t ex_cap = 0, snap0_cap = 0, snap1_cap = 0;
  int32_t* d_ex = nullptr;  // center | input | negs
  float *snap0 = nullptr, *snap1 = nullptr;

  // counters: [0] effective words, [1] examples, [2] raw words, [3] fault bits
  unsigned long long* d_counters = nullptr;

  // compute_loss: LOG_TABLE and the running loss ([0] double sum of the
  // parallel modes; the float32 running sum of SEQUENTIAL lives in [1])
  float* log_table = nullptr;
  double* d_loss = nullptr;
  unsigned int* d_queue = nullptr;  // k_sgns_atomic work queue (one counter)
  unsigned int* d_norm = nullptr;   // the stability cap's max squared row norm (float bits)
  int* d_waves = nullptr;           // waves that trained in the last Hogwild launch
  unsigned long long* d_stamps = nullptr;  // G2V_OPT_DEBUG_WRITE 8: segment cycle sums

  // replica merge: snapshot of both tables at the last merge, touched-row counts
  float *merge0 = nullptr, *merge1 = nullptr, *merge_cnt = nullptr;
  int64_t merge_ld = 0;
  bool merge_valid = false;
  // the merge's transport: RCCL (g2v_comm_init), an in-process group of
  // contexts (g2v_comm_init_local) or a host collective callback
  // (g2v_comm_init_host); the merge kernels are the same for all three
  int comm_kind = 0;  // kCommNone / kCommRccl / kCommLocal / kCommHost
  ncclComm_t comm = nullptr;
  g2v_local_group* lgroup = nullptr;
  g2v_collective_fn host_fn = nullptr;
  void* host_user = nullptr;
  float* h_coll = nullptr;  // pinned staging of the host transport
  size_t h_coll_cap = 0;
  int nranks = 1, rank = 0;
  int active_waves = 4;  // G2V_OPT_ACTIVE_WAVES
  int last_grid = 0, last_stripe_rows = 0, last_stripe_copies = 1, last_stripe2_rows = 0,
      last_stripe2_copies = 1;  // layout of the last Hogwild launch (g2v_stats)
  int last_tail0 = -1, last_tail1 = -1;  // its tail-store rows (-1: none)
  int64_t jobs = 0, launches = 0;

  // timing
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> t_sgns, t_samp;
};

// Hogwild staleness bound.  Every wave in flight holds one example whose
// updates the others do not see yet.  A row's share of the updates per
// example is u(r) = K * p_neg(r) (syn1neg, unigram^0.75 negatives) + p_tok(r)
// (its share of kept tokens: syn0 input and syn1neg centre); u_max = max_r.
// Too many waves x u_max and the sawtooth alpha restart diverges (round 2,
// C4 at 546, V 3,000 sample 0 at 315); well before
// that the Hogwild objective drifts from the sequential one (V 3,000, 200 k
// pairs, 3 iterations, 5 seeds: +0.4 % at 262-428, +0.05-0.1 % at 125-214).
// The pipelined kernel (G2V_OPT_ATOMIC_OVERLAP) reaches the atomic roof with
// 1 workgroup per CU at C2 and ~0.5 at C4, so the budget is set at the
// quiet end: waves x u_max <= 125 (C2 256 workgroups, C4 117, V 3,000 149).
constexpr double kStaleBudget = 125.0;

// Stability cap of the Hogwild waves (k_sgns_atomic, evaluated on the device
// before every launch).  The staleness budget above bounds the in-flight
// updates of the hottest syn1neg row; a hot syn0 row is the other risk: its
// delta sums K+1 terms g * syn1neg[t], so its in-flight updates overshoot once
// waves x p_tok x (K+1) x alpha x |syn1neg|^2 grows, which it does as
// training structures the vectors.  Measured, |syn1neg|^2 the
// largest squared row norm of syn1neg (a hot input's centres are any rows): a
// 3,000-gene corpus with planted modules at sample 0 diverged at a later
// sawtooth restart with 163 and 137 workgroups (a hot syn0 row's |v|^2 jumping
// 14 -> 90-215 and frozen there by the |f| >= 6 skip; products 190-250) and
// trained to the sequential order's objective at 64 (product 90); the C2 / C4
// vocabularies at sample 1e-3 and pure Zipf at sample 0 stay below the cap at
// their default grids.  So the waves that train are capped where the product,
// from |syn1neg|^2 just before the launch and the launch's largest alpha,
// reaches 100 (round 3 evaluated it once per g2v_train call, from a host
// read-back; a whole data-parallel epoch in one call was never re-capped).
constexpr double kSyn0Budget = 100.0;

// Cold-row plain stores (G2V_OPT_TAIL_STORE auto; k_sgns_atomic, DESIGN.md
// 5e).  A row whose update is a plain store of (row as read + delta) loses
// another wave's update when that wave writes it inside this wave's read-to-
// store window; waves x (the row's updates per example) estimates how many
// other in-flight examples hold it.  Auto: syn1neg rows from the first r with
// waves x u(r) <= this budget take stores (never a striped row); syn0 rows
// keep atomics.  C2 (1,024 waves): syn1neg from row ~7,700, 25 % of the
// syn1neg updates; corpora of <= ~5,000 genes have no syn1neg row this cold
// at their default grid.  Measured (profiles/r05): both tables
// from row 8,192 at C2 = +10.7 % pairs/s, 9.4 % of the stores lost an update
// (lost-update probe), the C2-vocabulary end-to-end gate at loss +0.38 %,
// objective +0.23 %, target function -0.43 % (atomics: +0.07 / -0.05 /
// -0.09 %); from 4,096 +12.4 %, 12 % lost, +0.58 / +0.42 / -0.63 %; from
// 2,048 the objective (+0.56 %) fails its 0.5 % bar.  syn0 rows by the same
// budget (p_tok(r), from row ~850 at C2, ~1,100 at 3,000-5,000 genes) took
// the dense 5,000-gene gate's target function from -0.46 to -0.84 % (1 %
// bar): syn0 holds the exported vectors, so it stays exact.
constexpr double kTailCollision = 0.15;

// Copies per striped hot row when G2V_OPT_STRIPE_COPIES is not set.  Every
// read of a striped row sums its copies (one more load batch on the example's
// critical path); every copy spreads that row's atomics.  At one workgroup per
// CU or more the kernel is bound by the memory-side atomics and 16 copies win
// (C2 266 WGs: 202.6 M ex/s vs 197.2 with 8).  Below, the grid is held down by
// the staleness budget and per-example latency binds: at D <= 256 the kernel
// loads all 15 extra copies in one batch (stripe_batch<1>, round 5), so 16
// copies cost no more latency than 8 and still spread the atomics (C2 sample 0
// at 162 WGs, round 5: 61.7 / 61.7 ms per launch vs 63.2 / 65.5 with 8); at
// D > 256 (batches of 7) 8 win (C4 at 121: 36.8 vs 36.1).
// the Hogwild grid of the launches being issued (the stability cap, DESIGN.md
// 5c, lowers the waves that train inside a launch, not the grid)
static int launch_grid(const g2v_ctx* c) { return c->sgns_grid; }

static int stripe_copies_eff(const g2v_ctx* c) {
  if (c->stripe_copies > 0) return c->stripe_copies;
  return (launch_grid(c) >= c->cus || c->nv == 1) ? 16 : 8;
}

// Second stripe tier when G2V_OPT_STRIPE2_ROWS is not set: rows up to 19 get 4
// copies each when the grid fills every CU (C2, interleaved A/B: 203.6 vs
// 200.3 M ex/s; 24 rows 203.0, 32 rows 202.0), none below, where per-example
// latency binds and the extra copy reads cost (C2 sample 0 at 162 WGs: 153.5
// vs 157.0; C4 at 121: 36.6 vs 36.7)
static int stripe2_rows_eff(const g2v_ctx* c) {
  if (c->stripe2_rows >= 0) return c->stripe2_rows;
  return launch_grid(c) >= c->cus ? 20 : 0;
}

// At most one workgroup per CU: C2 reaches the atomic roof there (266 vs 256
// workgroups: 203.6 vs 203.1 M examples/s), and the waves past it only add
// staleness -- on a 5,000-gene structured corpus the budget allowed 295 and
// the target function read -1.4 % against the sequential order, -0.97 % at
// 256
static int default_grid(int cus, int K, int nv, double u_max) {
  int g = std::min(cus * sgns_blocks_per_cu(K, nv), cus);
  if (u_max > 0.0) {
    const int waves = (int)(kStaleBudget / u_max);
    g = std::min(g, std::max(1, waves / (kSgnsThreads / 64)));
  }
  return g;
}

static int ctx_event(g2v_ctx* c, hipEvent_t* out) {
  if (c->ev_used == c->ev_pool.size()) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    c->ev_pool.push_back(e);
  }
  *out = c->ev_pool[c->ev_used++];
  return G2V_OK;
}

static int set_dev(g2v_ctx* c) {
  REQUIRE(c != nullptr, G2V_EINVAL, "null context");
  HIPCHK(hipSetDevice(c->device));
  return G2V_OK;
}

// ---------------------------------------------------------------------------
// RCCL, loaded at run time: a process that imported torch already holds
// torch's librccl.so.1 (same soname), and dlopen returns that copy, so the
// process has one RCCL; without torch the ROCm copy is loaded.
// ---------------------------------------------------------------------------
namespace {
struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclCommAbort) comm_abort = nullptr;  // optional
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string load_error;
  std::string library;  // what was dlopen()ed
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    // G2V_RCCL_LIB names another library with RCCL's entry points and nothing
    // else is tried (the test suite's stand-in, tests/rccl_standin/: two
    // ranks on ONE GPU, which real RCCL refuses as "Duplicate GPU").  It takes
    // effect only with the second opt-in G2V_ALLOW_RCCL_STANDIN=1, and says so
    // on stderr, so a stray variable cannot silently route real multi-GPU
    // merges through another library
    const char* over = getenv("G2V_RCCL_LIB");
    const char* allow = getenv("G2V_ALLOW_RCCL_STANDIN");
    if (over && *over && !(allow && std::string(allow) == "1")) {
      fprintf(stderr, "libg2v: ignoring G2V_RCCL_LIB=%s (set G2V_ALLOW_RCCL_STANDIN=1 to load it "
                      "instead of RCCL)\n", over);
      over = nullptr;
    }
    if (over && *over) {
      fprintf(stderr, "libg2v: G2V_RCCL_LIB=%s replaces RCCL for every merge of this process\n",
              over);
      h = dlopen(over, RTLD_NOW | RTLD_LOCAL);
      r.library = over;
    } else {
      for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
        if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL))) {
          r.library = name;
          break;
        }
    }
    if (!h) {
      const char* e = dlerror();
      r.load_error = std::string("dlopen(") + (over && *over ? over : "librccl.so.1") +
                     ") failed: " + (e ? e : "?");
      return;
    }
    bool ok = true;
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      ok = ok && fn != nullptr;
    };
    sym(r.get_unique_id, "ncclGetUniqueId");
    sym(r.comm_init_rank, "ncclCommInitRank");
    sym(r.comm_destroy, "ncclCommDestroy");
    sym(r.all_reduce, "ncclAllReduce");
    sym(r.broadcast, "ncclBroadcast");
    sym(r.group_start, "ncclGroupStart");
    sym(r.group_end, "ncclGroupEnd");
    sym(r.error_string, "ncclGetErrorString");
    if (!ok) {
      r.get_unique_id = nullptr;
      r.load_error = r.library + " lacks an nccl* entry point";
    }
    r.comm_abort = reinterpret_cast<decltype(&ncclCommAbort)>(dlsym(h, "ncclCommAbort"));
  });
  return r;
}

int rccl_fail(ncclResult_t e, const char* what) {
  const Rccl& r = rccl();
  return fail(G2V_ECOMM, "%s failed: %s", what, r.error_string ? r.error_string(e) : "?");
}
}  // namespace

#define NCCLCHK(x, what)                           \
  do {                                             \
    ncclResult_t e_ = (x);                         \
    if (e_ != ncclSuccess) return rccl_fail(e_, what); \
  } while (0)

// leave the current communicator (any transport) in an orderly way
static void comm_destroy(g2v_ctx* c) {
  if (c->comm && rccl().comm_destroy) (void)rccl().comm_destroy(c->comm);
  c->comm = nullptr;
  c->comm_kind = 0;
  c->lgroup = nullptr;
  c->host_fn = nullptr;
  c->host_user = nullptr;
  c->nranks = 1;
  c->rank = 0;
}

// device fault latched by the sampler (counters[3]); reads and clears it
static int check_fault(g2v_ctx* c) {
  unsigned long long f = 0;
  HIPCHK(hipMemcpy(&f, c->d_counters + 3, sizeof f, hipMemcpyDeviceToHost));
  if (!f) return G2V_OK;
  HIPCHK(hipMemset(c->d_counters + 3, 0, sizeof f));
  std::string m = "device corpus fault:";
  if (f & kFaultTokenRange) m += " token id outside [-1, V) (skipped as out of vocabulary);";
  if (f & kFaultJobSize) m += " job of several sentences holds > 10000 raw words (not trained);";
  return fail(G2V_EINVAL, "%s", m.c_str());
}

extern "C" {

const char* g2v_last_error(void) { return g_err.c_str(); }

int g2v_abi_version(void) { return G2V_ABI_VERSION; }

int g2v_create(int device, int32_t vocab_size, int32_t vector_size, int32_t negative,
               int32_t window, g2v_ctx** out) {
  REQUIRE(out != nullptr, G2V_EINVAL, "out is null");
  *out = nullptr;
  REQUIRE(vocab_size > 0, G2V_EINVAL, "vocab_size must be > 0 (got %d)", vocab_size);
  REQUIRE(vector_size >= 1 && vector_size <= G2V_MAX_DIM, G2V_EINVAL,
          "vector_size must be in [1, %d] (got %d)", G2V_MAX_DIM, vector_size);
  REQUIRE(window == 1, G2V_EINVAL,
          "window=%d: only window=1 (src/gene2vec.py:62) is implemented", window);
  const int nvec = (vector_size + 3) / 4;
  const int nv = nvec <= 64 ? 1 : 2;
  REQUIRE(sgns_supported(negative, nv), G2V_EINVAL,
          "negative=%d not compiled (supported: 1..20)", negative);
  // the update kernels address a table through one buffer resource (32-bit offsets)
  REQUIRE((int64_t)vocab_size * ((vector_size + 31) / 32 * 32) * 4 < ((int64_t)1 << 31),
          G2V_EINVAL, "vocab_size=%d x vector_size=%d exceeds the 2 GiB per-table limit",
          vocab_size, vector_size);
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  REQUIRE(device >= 0 && device < ndev, G2V_EINVAL, "device %d out of range (%d devices)", device,
          ndev);
  HIPCHK(hipSetDevice(device));

  g2v_ctx* c = new (std::nothrow) g2v_ctx();
  REQUIRE(c != nullptr, G2V_ENOMEM, "context allocation failed");
  c->device = device;
  c->V = vocab_size;
  c->D = vector_size;
  c->K = negative;
  c->window = window;
  c->nvec = nvec;
  c->nv = nv;
  c->ld = ((int64_t)vector_size + 31) / 32 * 32;  // 128-B aligned rows
  c->rec_stride = (3 + negative + 3) / 4 * 4;      // 16-B aligned records
  if (const char* s = getenv("G2V_SEG_JOBS")) c->seg_jobs = std::max(1, atoi(s));

  int rc = G2V_OK;
  auto bail = [&](int r) {
    g2v_destroy(c);
    return r;
  };
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess)
    return bail(fail(G2V_EHIP, "hipGetDeviceProperties failed"));
  c->cus = prop.multiProcessorCount;
  c->sgns_grid = default_grid(c->cus, negative, nv, 0.0);
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess)
    return bail(fail(G2V_EHIP, "hipStreamCreate failed"));
  c->stream = c->own_stream;
  if (hipEventCreateWithFlags(&c->stage_ev, hipEventDisableTiming) != hipSuccess)
    return bail(fail(G2V_EHIP, "hipEventCreate failed"));

  const size_t tab = (size_t)c->V * (size_t)c->ld;
  if (tab * sizeof(float) > 0x7fffffffull)
    return bail(fail(G2V_ERANGE, "table of %zu bytes exceeds the 2 GiB buffer-offset range", tab * 4));
  if ((rc = dev_alloc(&c->own0, tab)) || (rc = dev_alloc(&c->own1, tab)) ||
      (rc = dev_alloc(&c->lockf, (size_t)c->V)) || (rc = dev_alloc(&c->exp_table, kExpTableSize)) ||
      (rc = dev_alloc(&c->jump, 4 * (size_t)kJumpTab)) || (rc = dev_alloc(&c->cum, (size_t)c->V)) ||
      (rc = dev_alloc(&c->sample_int, (size_t)c->V)) ||
      (rc = dev_alloc(&c->bkt, (size_t)kBuckets + 1)) ||
      (rc = dev_alloc(&c->d_counts, (size_t)c->V)) || (rc = dev_alloc(&c->d_cpow, (size_t)c->V)) ||
      (rc = dev_alloc(&c->d_counters, 4)) || (rc = dev_alloc(&c->log_table, kExpTableSize)) ||
      (rc = dev_alloc(&c->d_loss, 2)) || (rc = dev_alloc(&c->d_queue, 1)) ||
      (rc = dev_alloc(&c->d_norm, 1)) || (rc = dev_alloc(&c->d_waves, 1)))
    return bail(rc);
  c->syn0 = c->own0;
  c->syn1 = c->own1;

  // constant tables: sigmoid LUT and LOG_TABLE ([ext] init(): LOG_TABLE[i] =
  // <REAL_t>log(EXP_TABLE[i])) and LCG jump tables, built on host
  float lut[kExpTableSize], logt[kExpTableSize];
  for (int i = 0; i < kExpTableSize; ++i) {
    const float x = ((float)i / (float)kExpTableSize * 2 - 1) * kMaxExp;
    const float e = (float)exp((double)x);
    lut[i] = e / (e + 1);
    logt[i] = (float)log((double)lut[i]);
  }
  std::vector<uint64_t> jt(4 * (size_t)kJumpTab);
  lcg_jump_tables(jt.data(), jt.data() + kJumpTab, jt.data() + 2 * kJumpTab,
                  jt.data() + 3 * kJumpTab);
  if (hipMemcpy(c->exp_table, lut, sizeof lut, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->log_table, logt, sizeof logt, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(c->d_loss, 0, 2 * sizeof(double)) != hipSuccess ||
      hipMemcpy(c->jump, jt.data(), jt.size() * sizeof(uint64_t), hipMemcpyHostToDevice) !=
          hipSuccess ||
      hipMemset(c->own0, 0, tab * sizeof(float)) != hipSuccess ||
      hipMemset(c->own1, 0, tab * sizeof(float)) != hipSuccess ||
      hipMemset(c->d_counters, 0, 4 * sizeof(unsigned long long)) != hipSuccess)
    return bail(fail(G2V_EHIP, "initial upload failed"));
  std::vector<float> ones((size_t)c->V, 1.0f);
  if (hipMemcpy(c->lockf, ones.data(), ones.size() * sizeof(float), hipMemcpyHostToDevice) !=
      hipSuccess)
    return bail(fail(G2V_EHIP, "lockf upload failed"));
  *out = c;
  return G2V_OK;
}

int g2v_destroy(g2v_ctx* c) {
  if (!c) return G2V_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  dev_free(c->own0);
  dev_free(c->own1);
  dev_free(c->lockf);
  dev_free(c->exp_table);
  dev_free(c->jump);
  dev_free(c->cum);
  dev_free(c->sample_int);
  dev_free(c->bkt);
  dev_free(c->d_counts);
  dev_free(c->d_cpow);
  dev_free(c->own_tok);
  dev_free(c->own_off);
  dev_free(c->d_job_sent);
  dev_free(c->d_job_alpha);
  dev_free(c->d_job_seed);
  if (c->side) (void)hipStreamSynchronize(c->side);
  dev_free(c->d_job_nex);
  dev_free(c->d_job_exoff);
  dev_free(c->d_rec);
  dev_free(c->d_job_nex2);
  dev_free(c->d_job_exoff2);
  dev_free(c->d_rec2);
  for (hipEvent_t e : {c->ev_up, c->ev_samp[0], c->ev_samp[1], c->ev_sgns[0], c->ev_sgns[1]})
    if (e) (void)hipEventDestroy(e);
  if (c->side) (void)hipStreamDestroy(c->side);
  dev_free(c->d_ex);
  dev_free(c->snap0);
  dev_free(c->snap1);
  dev_free(c->d_counters);
  dev_free(c->log_table);
  dev_free(c->d_loss);
  dev_free(c->d_queue);
  dev_free(c->d_norm);
  dev_free(c->d_waves);
  dev_free(c->d_stamps);
  dev_free(c->merge0);
  dev_free(c->merge1);
  dev_free(c->merge_cnt);
  comm_destroy(c);
  dev_free(c->stripe);
  dev_free(c->stripe2);
  dev_free(c->dbg16);
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  if (c->h_coll) (void)hipHostFree(c->h_coll);
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  if (c->stage_ev) (void)hipEventDestroy(c->stage_ev);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
  return G2V_OK;
}

int g2v_set_stream(g2v_ctx* c, void* s) {
  int rc = set_dev(c);
  if (rc) return rc;
  hipStream_t next = s ? (hipStream_t)s : c->own_stream;
  if (next != c->stream) {
    // the context's buffers are stream-ordered on one stream at a time: work
    // queued on the previous stream (and the side stream) finishes first
    if (c->stream) HIPCHK(hipStreamSynchronize(c->stream));
    if (c->side) HIPCHK(hipStreamSynchronize(c->side));
  }
  c->stream = next;
  return G2V_OK;
}

int g2v_set_option(g2v_ctx* c, int key, int64_t value) {
  int rc = set_dev(c);
  if (rc) return rc;
  switch (key) {
    case G2V_OPT_HOT_ROWS:
      REQUIRE(value >= -1 && value <= c->V, G2V_EINVAL, "hot_rows %lld out of [-1, V]",
              (long long)value);
      c->hot_rows = (int)value;
      return G2V_OK;
    case G2V_OPT_CACHE_POLICY:
      REQUIRE(value >= 0 && value <= 2, G2V_EINVAL, "cache policy %lld out of [0, 2]",
              (long long)value);
      c->cache_policy = (int)value;
      return G2V_OK;
    case G2V_OPT_SEG_JOBS:
      REQUIRE(value >= 1, G2V_EINVAL, "seg_jobs must be >= 1");
      c->seg_jobs = value;
      return G2V_OK;
    case G2V_OPT_TABLE_MEM: {
      // 0 hipMalloc (coarse-grained), 1 fine-grained, 2 uncached; contents reset to 0
      REQUIRE(value >= 0 && value <= 2, G2V_EINVAL, "table mem kind %lld out of [0, 2]",
              (long long)value);
      HIPCHK(hipStreamSynchronize(c->stream));
      const bool bound = c->syn0 != c->own0;
      dev_free(c->own0);
      dev_free(c->own1);
      const size_t bytes = sizeof(float) * (size_t)c->V * (size_t)(((int64_t)c->D + 31) / 32 * 32);
      const unsigned fl = value == 0 ? hipDeviceMallocDefault
                          : value == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached;
      HIPCHK(hipExtMallocWithFlags((void**)&c->own0, bytes, fl));
      HIPCHK(hipExtMallocWithFlags((void**)&c->own1, bytes, fl));
      HIPCHK(hipMemset(c->own0, 0, bytes));
      HIPCHK(hipMemset(c->own1, 0, bytes));
      if (!bound) {
        c->syn0 = c->own0;
        c->syn1 = c->own1;
      }
      return G2V_OK;
    }
    case G2V_OPT_STRIPE_ROWS:
      REQUIRE(value >= 0 && value <= 65536, G2V_EINVAL, "stripe rows out of [0, 65536]");
      c->stripe_rows = (int)value;
      return G2V_OK;
    case G2V_OPT_STRIPE2_ROWS:
      REQUIRE(value >= -1 && value <= (1 << 20), G2V_EINVAL,
              "second-tier stripe rows out of range");
      c->stripe2_rows = (int)value;  // -1: auto (stripe2_rows_eff)
      return G2V_OK;
    case G2V_OPT_STRIPE2_COPIES:
      REQUIRE(value == 2 || value == 4 || value == 8, G2V_EINVAL,
              "second-tier stripe copies must be 2, 4 or 8");
      c->stripe2_copies = (int)value;
      return G2V_OK;
    case G2V_OPT_STRIPE_COPIES:
      REQUIRE(value >= 0 && value <= 32, G2V_EINVAL, "stripe copies out of [0, 32]");
      c->stripe_copies = (int)value;  // explicit: no longer chosen from the grid
      return G2V_OK;
    case G2V_OPT_DEBUG_WRITE: {
      // 2 (gather roof) and 8 (stamps) are compiled for the reference's shape
      // only (negative 5, D <= 256); the other modes only into the ablation
      // build (-DG2V_ABLATIONS).  Refused otherwise instead of silently
      // running the production kernel.
#ifdef G2V_ABLATIONS
      const bool known = value >= 0 && value <= 10;
#else
      const bool known = value == 0 || value == 2 || value == 8;
#endif
      REQUIRE(known, G2V_EINVAL, "debug write mode %lld is not compiled into this library",
              (long long)value);
#ifdef G2V_ABLATIONS
      // the lost-update probe also at the C4 shape (negative 15, D 257..512)
      if (value == 10 && c->K == 15 && c->nv == 2) {
        c->debug_write = 10;
        return G2V_OK;
      }
#endif
      REQUIRE(value == 0 || (c->K == 5 && c->nv == 1), G2V_EINVAL,
              "debug write mode %lld needs negative 5 and vector_size <= 256 (have %d, %d)",
              (long long)value, c->K, c->D);
      c->debug_write = (int)value;
      return G2V_OK;
    }
    case G2V_OPT_ATOMIC_OVERLAP:
      REQUIRE(value == 0 || value == 1, G2V_EINVAL, "atomic overlap must be 0 or 1");
      c->atomic_overlap = (int)value;
      return G2V_OK;
    case G2V_OPT_SAMPLE_OVERLAP:
      REQUIRE(value == 0 || value == 1, G2V_EINVAL, "sample overlap must be 0 or 1");
      c->sample_overlap = (int)value;
      return G2V_OK;
    case G2V_OPT_MERGE_EVERY_JOBS:
      REQUIRE(value >= 0, G2V_EINVAL, "merge cadence must be >= 0");
      c->merge_every = value;
      return G2V_OK;
    case G2V_OPT_MERGE_RULE:
      REQUIRE(value == G2V_MERGE_TOUCH || value == G2V_MERGE_MEAN || value == G2V_MERGE_ALIGN,
              G2V_EINVAL, "merge rule %lld", (long long)value);
      c->merge_rule = (int)value;
      return G2V_OK;
    case G2V_OPT_GRID:
      REQUIRE(value >= 0, G2V_EINVAL, "grid must be >= 0");
      c->grid_user = value > 0;
      c->sgns_grid = value > 0 ? (int)value : default_grid(c->cus, c->K, c->nv, c->u_max);
      return G2V_OK;
    case G2V_OPT_MERGE_BETA_MILLI:
      REQUIRE(value >= 0 && value <= 4000, G2V_EINVAL, "merge beta (x1000) out of [0, 4000]");
      c->merge_beta = (float)value / 1000.0f;
      return G2V_OK;
    case G2V_OPT_MERGE_GAMMA_MILLI:
      REQUIRE(value >= 250 && value <= 16000, G2V_EINVAL,
              "merge gamma (x1000) out of [250, 16000]");
      c->merge_gamma = (float)value / 1000.0f;
      return G2V_OK;
    case G2V_OPT_RETIRED_19:
    case G2V_OPT_RETIRED_20:
      return fail(G2V_EINVAL, "option %d was retired in ABI 5 (measured slower, DESIGN.md 5d)",
                  key);
    case G2V_OPT_TAIL_STORE:
      REQUIRE(value >= -1 && value <= c->V, G2V_EINVAL, "tail store row %lld out of [-1, V]",
              (long long)value);
      c->tail_store = (int)value;
      return G2V_OK;
    case G2V_OPT_DEBUG_FAIL_MERGE:
      REQUIRE(value >= 0, G2V_EINVAL, "debug fail merge < 0");
      c->debug_fail_merge = value;
      return G2V_OK;
    case G2V_OPT_ACTIVE_WAVES:
      REQUIRE(value >= 1 && value <= kSgnsThreads / 64, G2V_EINVAL, "active waves out of [1, %d]",
              kSgnsThreads / 64);
      c->active_waves = (int)value;
      return G2V_OK;
    default:
      return fail(G2V_EINVAL, "unknown option key %d", key);
  }
}

int g2v_get_option(g2v_ctx* c, int key, int64_t* out) {
  REQUIRE(c && out, G2V_EINVAL, "null argument");
  switch (key) {
    case G2V_OPT_HOT_ROWS: *out = c->hot_rows; return G2V_OK;
    case G2V_OPT_CACHE_POLICY: *out = c->cache_policy; return G2V_OK;
    case G2V_OPT_SEG_JOBS: *out = c->seg_jobs; return G2V_OK;
    case G2V_OPT_GRID: *out = c->sgns_grid; return G2V_OK;
    case G2V_OPT_DEBUG_WRITE: *out = c->debug_write; return G2V_OK;
    case G2V_OPT_STRIPE_ROWS: *out = c->stripe_rows; return G2V_OK;
    case G2V_OPT_STRIPE_COPIES: *out = stripe_copies_eff(c); return G2V_OK;
    case G2V_OPT_STRIPE2_ROWS: *out = stripe2_rows_eff(c); return G2V_OK;
    case G2V_OPT_STRIPE2_COPIES: *out = c->stripe2_copies; return G2V_OK;
    case G2V_OPT_ATOMIC_OVERLAP: *out = c->atomic_overlap; return G2V_OK;
    case G2V_OPT_SAMPLE_OVERLAP: *out = c->sample_overlap; return G2V_OK;
    case G2V_OPT_MERGE_EVERY_JOBS: *out = c->merge_every; return G2V_OK;
    case G2V_OPT_MERGE_RULE: *out = c->merge_rule; return G2V_OK;
    case G2V_OPT_ACTIVE_WAVES: *out = c->active_waves; return G2V_OK;
    case G2V_OPT_MERGE_BETA_MILLI: *out = (int64_t)lrintf(c->merge_beta * 1000.0f); return G2V_OK;
    case G2V_OPT_MERGE_GAMMA_MILLI: *out = (int64_t)lrintf(c->merge_gamma * 1000.0f); return G2V_OK;
    case G2V_OPT_DEBUG_FAIL_MERGE: *out = c->debug_fail_merge; return G2V_OK;
    case G2V_OPT_TAIL_STORE: *out = c->tail_store; return G2V_OK;
    default: return fail(G2V_EINVAL, "option key %d cannot be read", key);
  }
}

int g2v_row_stride(g2v_ctx* c, int64_t* ld_out) {
  REQUIRE(c && ld_out, G2V_EINVAL, "null argument");
  *ld_out = c->ld;
  return G2V_OK;
}

int g2v_set_vocab(g2v_ctx* c, const int64_t* counts, double sample, double ns_exponent,
                  uint32_t* cum_out, uint32_t* sample_int_out) {
  int rc = set_dev(c);
  if (rc) return rc;
  REQUIRE(counts != nullptr, G2V_EINVAL, "counts is null");
  REQUIRE(sample >= 0.0, G2V_EINVAL, "sample must be >= 0");
  for (int32_t i = 0; i < c->V; ++i)
    REQUIRE(counts[i] > 0, G2V_EINVAL, "counts[%d] = %lld must be > 0", i, (long long)counts[i]);
  {
    // staleness budget of the Hogwild grid (default_grid): u(r) = K p_neg(r) +
    // p_tok(r), p_tok from the downsampled counts (launch_vocab's keep rule)
    double zn = 0.0, zt = 0.0, total = 0.0;
    std::vector<double> pn((size_t)c->V), pt((size_t)c->V);
    for (int32_t i = 0; i < c->V; ++i) total += (double)counts[i];
    double thr = total;
    if (sample > 0.0 && sample < 1.0) thr = sample * total;
    else if (sample >= 1.0) thr = (double)(int64_t)(sample * (3.0 + sqrt(5.0)) / 2.0);
    for (int32_t i = 0; i < c->V; ++i) {
      const double v = (double)counts[i];
      pn[i] = pow(v, ns_exponent);
      zn += pn[i];
      pt[i] = v * std::min(1.0, (sqrt(v / thr) + 1.0) * (thr / v));
      zt += pt[i];
    }
    double um = 0.0, pm = 0.0;
    for (int32_t i = 0; i < c->V; ++i) {
      um = std::max(um, c->K * pn[i] / zn + pt[i] / zt);
      pm = std::max(pm, pt[i] / zt);
    }
    c->u_max = um;
    c->p_tok_max = pm;
    c->u_row.resize((size_t)c->V);
    double suffix = 0.0;
    for (int32_t i = c->V - 1; i >= 0; --i) {
      suffix = std::max(suffix, c->K * pn[i] / zn + pt[i] / zt);
      c->u_row[i] = suffix;
    }
    if (!c->grid_user) c->sgns_grid = default_grid(c->cus, c->K, c->nv, um);
  }
  HIPCHK(hipMemcpyAsync(c->d_counts, counts, sizeof(int64_t) * c->V, hipMemcpyHostToDevice,
                        c->stream));
  HIPCHK(launch_vocab(c->d_counts, c->d_cpow, c->V, ns_exponent, sample, c->cum, c->sample_int,
                      c->bkt, c->stream));
  c->sample_on = sample != 0.0;
  if (cum_out)
    HIPCHK(hipMemcpyAsync(cum_out, c->cum, sizeof(uint32_t) * c->V, hipMemcpyDeviceToHost,
                          c->stream));
  if (sample_int_out)
    HIPCHK(hipMemcpyAsync(sample_int_out, c->sample_int, sizeof(uint32_t) * c->V,
                          hipMemcpyDeviceToHost, c->stream));
  if (cum_out || sample_int_out) {
    HIPCHK(hipStreamSynchronize(c->stream));
    if (cum_out && cum_out[c->V - 1] != 2147483647u)
      return fail(G2V_EINVAL, "cum_table[-1] = %u != 2**31-1", cum_out[c->V - 1]);
  }
  c->vocab_ready = true;
  return G2V_OK;
}

int g2v_bind_tables(g2v_ctx* c, float* s0, float* s1, int64_t ld) {
  int rc = set_dev(c);
  if (rc) return rc;
  if (!s0 && !s1) {
    c->syn0 = c->own0;
    c->syn1 = c->own1;
    c->ld = ((int64_t)c->D + 31) / 32 * 32;
    return G2V_OK;
  }
  REQUIRE(s0 && s1, G2V_EINVAL, "bind both tables or neither");
  REQUIRE(ld >= c->D && ld % 4 == 0, G2V_EINVAL, "ld=%lld must be >= D=%d and a multiple of 4",
          (long long)ld, c->D);
  REQUIRE(((uintptr_t)s0 % 16) == 0 && ((uintptr_t)s1 % 16) == 0, G2V_EINVAL,
          "tables must be 16-byte aligned");
  // the update kernels address a table through one buffer resource (32-bit
  // offsets): rows past 2 GiB would read as zeros and lane offsets would wrap
  REQUIRE((int64_t)c->V * ld * 4 < ((int64_t)1 << 31), G2V_ERANGE,
          "vocab_size=%d x ld=%lld exceeds the 2 GiB per-table limit", c->V, (long long)ld);
  c->syn0 = s0;
  c->syn1 = s1;
  c->ld = ld;
  c->weights_ready = true;
  if (c->merge_valid) return g2v_merge_snapshot(c);
  return G2V_OK;
}

int g2v_set_weights(g2v_ctx* c, const float* s0, const float* s1, const float* lockf) {
  int rc = set_dev(c);
  if (rc) return rc;
  const size_t row = sizeof(float) * (size_t)c->D, pitch = sizeof(float) * (size_t)c->ld;
  if (s0) {
    HIPCHK(hipMemsetAsync(c->syn0, 0, pitch * c->V, c->stream));
    HIPCHK(hipMemcpy2DAsync(c->syn0, pitch, s0, row, row, c->V, hipMemcpyHostToDevice, c->stream));
  }
  if (s1) {
    HIPCHK(hipMemsetAsync(c->syn1, 0, pitch * c->V, c->stream));
    HIPCHK(hipMemcpy2DAsync(c->syn1, pitch, s1, row, row, c->V, hipMemcpyHostToDevice, c->stream));
  }
  if (lockf)
    HIPCHK(hipMemcpyAsync(c->lockf, lockf, sizeof(float) * c->V, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));  // host buffers are only borrowed for the call
  c->weights_ready = true;
  if (c->merge_valid) return g2v_merge_snapshot(c);
  return G2V_OK;
}

int g2v_get_weights(g2v_ctx* c, float* s0, float* s1) {
  int rc = set_dev(c);
  if (rc) return rc;
  const size_t row = sizeof(float) * (size_t)c->D, pitch = sizeof(float) * (size_t)c->ld;
  if (s0)
    HIPCHK(hipMemcpy2DAsync(s0, row, c->syn0, pitch, row, c->V, hipMemcpyDeviceToHost, c->stream));
  if (s1)
    HIPCHK(hipMemcpy2DAsync(s1, row, c->syn1, pitch, row, c->V, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return G2V_OK;
}

}  // extern "C"

// min / max of n int32 ids (host corpus check, parallel over up to 8 threads)
static void id_range(const int32_t* x, int64_t n, int32_t* lo, int32_t* hi) {
  const int64_t kGrain = 1 << 22;
  const int nt = (int)std::min<int64_t>(8, std::max<int64_t>(1, n / kGrain));
  std::vector<int32_t> mn(nt, INT32_MAX), mx(nt, INT32_MIN);
  auto run = [&](int k) {
    const int64_t b = n * k / nt, e = n * (k + 1) / nt;
    int32_t a = INT32_MAX, z = INT32_MIN;
    for (int64_t i = b; i < e; ++i) {
      a = std::min(a, x[i]);
      z = std::max(z, x[i]);
    }
    mn[k] = a;
    mx[k] = z;
  };
  std::vector<std::thread> th;
  for (int k = 1; k < nt; ++k) th.emplace_back(run, k);
  run(0);
  for (auto& t : th) t.join();
  *lo = *std::min_element(mn.begin(), mn.end());
  *hi = *std::max_element(mx.begin(), mx.end());
}

extern "C" {

int g2v_set_corpus(g2v_ctx* c, const int32_t* tokens, int64_t n_tokens, const int64_t* sent_off,
                   int64_t n_sent, int64_t sent_len, uint32_t flags) {
  int rc = set_dev(c);
  if (rc) return rc;
  REQUIRE(n_tokens >= 0 && n_sent >= 0, G2V_EINVAL, "negative sizes");
  REQUIRE(tokens || n_tokens == 0, G2V_EINVAL, "tokens is null");
  REQUIRE(sent_len > 0 || sent_off, G2V_EINVAL, "need sent_off or sent_len > 0");
  if (sent_len > 0)
    REQUIRE(n_tokens == n_sent * sent_len, G2V_EINVAL,
            "n_tokens=%lld != n_sent*sent_len=%lld", (long long)n_tokens,
            (long long)(n_sent * sent_len));
  HIPCHK(hipStreamSynchronize(c->stream));
  dev_free(c->own_tok);
  dev_free(c->own_off);
  c->h_sent_off.clear();
  c->n_tok = n_tokens;
  c->n_sent = n_sent;
  c->sent_len = sent_len;
  if (flags & G2V_CORPUS_DEVICE) {
    c->tok = tokens;
    c->sent_off = sent_len > 0 ? nullptr : sent_off;
  } else {
    if (n_tokens > 0) {
      int32_t lo, hi;
      id_range(tokens, n_tokens, &lo, &hi);
      REQUIRE(lo >= -1 && hi < c->V, G2V_EINVAL,
              "corpus ids must lie in [-1, V=%d) (found [%d, %d])", c->V, lo, hi);
    }
    if (sent_len <= 0) {
      REQUIRE(sent_off[0] == 0 && sent_off[n_sent] == n_tokens, G2V_EINVAL,
              "sent_off must start at 0 and end at n_tokens");
      for (int64_t i = 0; i < n_sent; ++i)
        REQUIRE(sent_off[i + 1] >= sent_off[i], G2V_EINVAL, "sent_off decreases at %lld",
                (long long)i);
    }
    if ((rc = dev_alloc(&c->own_tok, (size_t)n_tokens))) return rc;
    HIPCHK(hipMemcpy(c->own_tok, tokens, sizeof(int32_t) * n_tokens, hipMemcpyHostToDevice));
    c->tok = c->own_tok;
    if (sent_len > 0) {
      c->sent_off = nullptr;
    } else {
      if ((rc = dev_alloc(&c->own_off, (size_t)n_sent + 1))) return rc;
      HIPCHK(hipMemcpy(c->own_off, sent_off, sizeof(int64_t) * (n_sent + 1),
                       hipMemcpyHostToDevice));
      c->sent_off = c->own_off;
      c->h_sent_off.assign(sent_off, sent_off + n_sent + 1);
    }
  }
  c->corpus_ready = true;
  return G2V_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// training driver
// ---------------------------------------------------------------------------
static int64_t tokens_between(const g2v_ctx* c, int64_t s0, int64_t s1) {
  if (c->sent_len > 0) return (s1 - s0) * c->sent_len;
  if (!c->h_sent_off.empty()) return c->h_sent_off[s1] - c->h_sent_off[s0];
  return -1;  // unknown on host (device-borrowed CSR)
}

// stage job tables through pinned memory so the copy is truly asynchronous
static int upload_jobs(g2v_ctx* c, const int64_t* job_sent, const float* job_alpha,
                       const uint64_t* job_seed, int64_t n_jobs) {
  int rc;
  if ((rc = dev_reserve(c->stream, &c->d_job_sent, &c->job_cap, n_jobs + 1))) return rc;
  if ((rc = dev_reserve(c->stream, &c->d_job_alpha, &c->job_alpha_cap, std::max<int64_t>(n_jobs, 1))))
    return rc;
  if ((rc = dev_reserve(c->stream, &c->d_job_seed, &c->job_seed_cap, std::max<int64_t>(n_jobs, 1))))
    return rc;
  const size_t b_sent = sizeof(int64_t) * (n_jobs + 1), b_alpha = sizeof(float) * n_jobs,
               b_seed = sizeof(uint64_t) * n_jobs;
  const size_t need = b_sent + b_seed + b_alpha + 64;
  if (c->stage_pending) {
    HIPCHK(hipEventSynchronize(c->stage_ev));
    c->stage_pending = false;
  }
  if (need > c->h_stage_cap) {
    if (c->h_stage) HIPCHK(hipHostFree(c->h_stage));
    c->h_stage = nullptr;
    HIPCHK(hipHostMalloc(&c->h_stage, need * 2, hipHostMallocDefault));
    c->h_stage_cap = need * 2;
  }
  char* p = (char*)c->h_stage;
  memcpy(p, job_sent, b_sent);
  memcpy(p + b_sent, job_seed, b_seed);
  if (job_alpha) memcpy(p + b_sent + b_seed, job_alpha, b_alpha);
  else memset(p + b_sent + b_seed, 0, b_alpha);
  HIPCHK(hipMemcpyAsync(c->d_job_sent, p, b_sent, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_job_seed, p + b_sent, b_seed, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_job_alpha, p + b_sent + b_seed, b_alpha, hipMemcpyHostToDevice,
                        c->stream));
  HIPCHK(hipEventRecord(c->stage_ev, c->stream));
  c->stage_pending = true;
  return G2V_OK;
}

static int check_jobs(const g2v_ctx* c, const int64_t* job_sent, int64_t n_jobs) {
  REQUIRE(n_jobs >= 0, G2V_EINVAL, "n_jobs < 0");
  REQUIRE(job_sent != nullptr, G2V_EINVAL, "job_sent is null");
  for (int64_t j = 0; j < n_jobs; ++j) {
    REQUIRE(job_sent[j] >= 0 && job_sent[j] <= job_sent[j + 1] && job_sent[j + 1] <= c->n_sent,
            G2V_EINVAL, "job %lld sentence range [%lld, %lld) invalid (n_sent=%lld)",
            (long long)j, (long long)job_sent[j], (long long)job_sent[j + 1],
            (long long)c->n_sent);
    // [ext] _job_producer gives a sentence over batch_words a job of its own;
    // train_batch_sg truncates it at 10000 effective words
    const int64_t nt = tokens_between(c, job_sent[j], job_sent[j + 1]);
    REQUIRE(nt <= kBatchWords || job_sent[j + 1] - job_sent[j] == 1, G2V_ERANGE,
            "job %lld holds %lld raw words in %lld sentences > batch_words %d", (long long)j,
            (long long)nt, (long long)(job_sent[j + 1] - job_sent[j]), kBatchWords);
  }
  return G2V_OK;
}

// count -> scan -> write records for jobs [j0, j0+nj); returns the record buffer
static int sample_segment(g2v_ctx* c, int64_t j0, int64_t nj, bool timing, int buf = 0,
                          hipStream_t st = nullptr) {
  int rc;
  if (!st) st = c->stream;
  int32_t*& nex = buf ? c->d_job_nex2 : c->d_job_nex;
  int64_t*& exoff = buf ? c->d_job_exoff2 : c->d_job_exoff;
  int32_t*& rec = buf ? c->d_rec2 : c->d_rec;
  int64_t& nex_cap = buf ? c->nex_cap2 : c->nex_cap;
  int64_t& exoff_cap = buf ? c->exoff_cap2 : c->exoff_cap;
  int64_t& rec_cap = buf ? c->rec_cap2 : c->rec_cap;
  // a buffer that must grow is freed after its last reader (the training
  // stream) and the side stream are idle
  if (c->side && (nj > nex_cap || nj + 1 > exoff_cap)) HIPCHK(hipStreamSynchronize(c->side));
  if ((rc = dev_reserve(c->stream, &nex, &nex_cap, nj))) return rc;
  if ((rc = dev_reserve(c->stream, &exoff, &exoff_cap, nj + 1))) return rc;
  // examples per job <= 2 * raw words (window 1)
  int64_t max_ex = nj * 2 * (int64_t)kBatchWords;
  // tighter bound when the token count is known on host
  // (job_sent lives in pinned staging, still valid: read it from there)
  const int64_t* hjs = (const int64_t*)c->h_stage;
  const int64_t tk = tokens_between(c, hjs[j0], hjs[j0 + nj]);
  if (tk >= 0) max_ex = std::max<int64_t>(2 * std::min<int64_t>(tk, nj * (int64_t)kBatchWords), 1);
  if (c->side && max_ex * c->rec_stride > rec_cap) HIPCHK(hipStreamSynchronize(c->side));
  if ((rc = dev_reserve(c->stream, &rec, &rec_cap, max_ex * c->rec_stride))) return rc;

  SampleArgs a{};
  a.tok = c->tok;
  a.sent_off = c->sent_off;
  a.sent_len = c->sent_len;
  a.job_sent = c->d_job_sent;
  a.job_seed = c->d_job_seed;
  a.job_alpha = c->d_job_alpha;
  a.job0 = j0;
  a.sample_int = c->sample_int;
  a.sample_on = c->sample_on;
  a.cum = c->cum;
  a.bkt = c->bkt;
  a.V = c->V;
  a.jump = LcgJump{c->jump, c->jump + kJumpTab, c->jump + 2 * kJumpTab, c->jump + 3 * kJumpTab};
  a.K = c->K;
  a.rec_stride = c->rec_stride;
  a.job_nex = nex;
  a.job_exoff = exoff;
  a.rec = rec;
  a.counters = c->d_counters;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (timing) {
    if ((rc = ctx_event(c, &e0)) || (rc = ctx_event(c, &e1))) return rc;
    HIPCHK(hipEventRecord(e0, st));
  }
  HIPCHK(launch_job_sample(false, a, nj, st));
  HIPCHK(launch_scan_jobs(nex, nj, exoff, c->d_counters + 1, st));
  HIPCHK(launch_job_sample(true, a, nj, st));
  if (timing) {
    HIPCHK(hipEventRecord(e1, st));
    c->t_samp.emplace_back(e0, e1);
  }
  return G2V_OK;
}

// amax: the launch's largest alpha, for the stability cap of a Hogwild
// launch on the library's grid (0: no cap)
static int run_sgns(g2v_ctx* c, const int64_t* n_examples_dev, int mode, bool timing,
                    bool closs, const float* rd0, const float* rd1,
                    const int32_t* rec = nullptr, float amax = 0.f) {
  SgnsArgs s{};
  s.rec = rec ? rec : c->d_rec;
  s.rec_stride = c->rec_stride;
  s.n_examples = n_examples_dev;
  s.rd0 = rd0;
  s.rd1 = rd1;
  s.wr0 = c->syn0;
  s.wr1 = c->syn1;
  s.lockf = c->lockf;
  s.ld = c->ld;
  s.nvec = c->nvec;
  s.D = c->D;
  s.V = c->V;
  s.hot_rows = c->hot_rows < 0 ? c->V : std::min(c->hot_rows, c->V);
  s.exp_table = c->exp_table;
  // 6: production writes, 7: scratch atomics (mode 4); both read main rows only
  s.debug_write = c->debug_write == 6 ? 0 : c->debug_write == 7 ? 4 : c->debug_write;
  s.skip_copy_reads = (c->debug_write == 6 || c->debug_write == 7) ? 1 : 0;
  s.compute_loss = closs ? 1 : 0;
  s.log_table = c->log_table;
  s.loss_f64 = c->d_loss;
  s.loss_f32 = reinterpret_cast<float*>(c->d_loss + 1);
  const bool atomic_kernel = mode == kModeHogwild && s.hot_rows >= c->V;
  const int copies = stripe_copies_eff(c);
  // rows past what a 1 GiB stripe buffer holds stay unstriped (kStripeMaxBytes)
  const int64_t max_rows =
      copies > 1 ? kStripeMaxBytes / (2 * 4 * (int64_t)(copies - 1) * c->ld) : 0;
  const int srows = (int)std::min<int64_t>(std::min(c->stripe_rows, c->V), max_rows);
  const bool striped = atomic_kernel && copies > 1 && srows > 0;
  s.stripe_rows = striped ? srows : 0;
  s.stripe_copies = striped ? copies : 1;
  s.overlap = c->atomic_overlap;
  s.active_waves = c->active_waves;
  s.queue = c->d_queue;
  int rc;
  if (striped) {
    const int64_t need = 2 * (int64_t)(s.stripe_copies - 1) * s.stripe_rows * c->ld;
    if (need > c->stripe_cap) {
      if ((rc = dev_reserve(c->stream, &c->stripe, &c->stripe_cap, need))) return rc;
      HIPCHK(hipMemsetAsync(c->stripe, 0, sizeof(float) * c->stripe_cap, c->stream));
    }
  }
  s.stripe = c->stripe;
  // second tier (not in the ablation builds, which address only the first)
  const int64_t max_rows2 = kStripeMaxBytes / (2 * 4 * (int64_t)(c->stripe2_copies - 1) * c->ld);
  const int r2 = (int)std::min<int64_t>(std::min(stripe2_rows_eff(c), c->V),
                                        (int64_t)s.stripe_rows + max_rows2);
  const bool tier2 = striped &&
                     (c->debug_write == 0 || c->debug_write == 6 || c->debug_write == 8 ||
                      c->debug_write == 9 || c->debug_write == 10) &&
                     r2 > s.stripe_rows;
  s.stripe2_rows = tier2 ? r2 : s.stripe_rows;
  s.stripe2_copies = tier2 ? c->stripe2_copies : 1;
  if (tier2) {
    const int64_t need = 2 * (int64_t)(c->stripe2_copies - 1) * (r2 - s.stripe_rows) * c->ld;
    if (need > c->stripe2_cap) {
      if ((rc = dev_reserve(c->stream, &c->stripe2, &c->stripe2_cap, need))) return rc;
      HIPCHK(hipMemsetAsync(c->stripe2, 0, sizeof(float) * c->stripe2_cap, c->stream));
    }
  }
  s.stripe2 = c->stripe2;
  // cold-row plain stores (G2V_OPT_TAIL_STORE), never on a striped row
  s.tail_row0 = s.tail_row1 = 0x7fffffff;
  if (atomic_kernel && (c->debug_write == 0 || c->debug_write == 8 || c->debug_write == 10) &&
      c->tail_store != 0) {
    int t0 = c->tail_store, t1 = c->tail_store;
    if (c->tail_store < 0 && c->active_waves < kSgnsThreads / 64) {
      t0 = t1 = c->V;  // auto is off in the one-wave parity mode (G2V_OPT_ACTIVE_WAVES)
    } else if (c->tail_store < 0) {
      // auto: the collision budget over the waves this launch may run; the
      // first row from which every later row is under it (u_row is a suffix
      // max: a negative ns_exponent or unsorted counts put hot rows late)
      const double waves = (double)launch_grid(c) * c->active_waves;
      auto first_under = [&](const std::vector<double>& rate) {
        return (int)(std::partition_point(rate.begin(), rate.end(),
                                          [&](double x) { return waves * x > kTailCollision; }) -
                     rate.begin());
      };
      t1 = c->u_row.empty() ? c->V : first_under(c->u_row);
      t0 = c->V;  // syn0 (the exported vectors) keeps atomics: see kTailCollision
    }
    const int floor_row = std::max(s.stripe_rows, s.stripe2_rows);
    if (t0 < c->V) s.tail_row0 = std::max(t0, floor_row);
    if (t1 < c->V) s.tail_row1 = std::max(t1, floor_row);
  }
  if (c->debug_write == 3 || c->debug_write == 4 || c->debug_write == 7) {
    const int64_t rows = (int64_t)c->V + (int64_t)(s.stripe_copies - 1) * s.stripe_rows;
    const int64_t words = rows * c->ld * (c->debug_write == 3 ? 1 : 2);
    if ((rc = dev_reserve(c->stream, &c->dbg16, &c->dbg16_cap, words))) return rc;
    HIPCHK(hipMemsetAsync(c->dbg16, 0, sizeof(uint32_t) * c->dbg16_cap, c->stream));
  }
  s.dbg16 = c->dbg16;
  if ((c->debug_write == 8 || c->debug_write == 10) && !c->d_stamps) {
    if ((rc = dev_alloc(&c->d_stamps, kStampWords))) return rc;
    HIPCHK(hipMemsetAsync(c->d_stamps, 0, kStampWords * sizeof(unsigned long long), c->stream));
  }
  s.stamps = c->d_stamps;
  s.waves_out = atomic_kernel ? c->d_waves : nullptr;
  if (atomic_kernel && amax > 0.f && !c->grid_user) {
    // the cap from the tables as they are now (every launch: a single long
    // call -- a data-parallel epoch -- is re-capped as the norms grow), with
    // no host synchronisation; 33 us at C2 per ~28 ms launch
    HIPCHK(hipMemsetAsync(c->d_norm, 0, sizeof(unsigned int), c->stream));
    HIPCHK(launch_row_norm2_max(c->syn1, c->V, c->ld, c->D, c->d_norm, c->stream));
    s.norm_bits = c->d_norm;
    s.cap_coef = (float)(c->p_tok_max * (c->K + 1) * (double)amax);
    s.cap_budget = (float)kSyn0Budget;
  }
  if (atomic_kernel) HIPCHK(hipMemsetAsync(c->d_queue, 0, sizeof(unsigned int), c->stream));
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (timing) {
    if ((rc = ctx_event(c, &e0)) || (rc = ctx_event(c, &e1))) return rc;
    HIPCHK(hipEventRecord(e0, c->stream));
  }
  HIPCHK(launch_sgns(s, c->K, c->nv, mode, c->cache_policy, launch_grid(c), c->stream));
  HIPCHK(launch_fold_stripes(c->syn0, c->syn1, c->stripe, s.stripe_rows, s.stripe_copies, c->ld,
                             c->nvec, c->stream));
  if (tier2)
    HIPCHK(launch_fold_stripes(c->syn0 + (int64_t)s.stripe_rows * c->ld,
                               c->syn1 + (int64_t)s.stripe_rows * c->ld, c->stripe2,
                               s.stripe2_rows - s.stripe_rows, s.stripe2_copies, c->ld, c->nvec,
                               c->stream));
  if (timing) {
    HIPCHK(hipEventRecord(e1, c->stream));
    c->t_sgns.emplace_back(e0, e1);
  }
  if (atomic_kernel) {
    c->last_grid = launch_grid(c);
    c->last_stripe_rows = s.stripe_rows;
    c->last_stripe_copies = s.stripe_copies;
    c->last_stripe2_rows = s.stripe2_rows;
    c->last_stripe2_copies = s.stripe2_copies;
    c->last_tail0 = s.tail_row0 < c->V ? s.tail_row0 : -1;
    c->last_tail1 = s.tail_row1 < c->V ? s.tail_row1 : -1;
  }
  c->launches++;
  return G2V_OK;
}

static int merge_now(g2v_ctx* c, int rule);
static int comm_broadcast_tables(g2v_ctx* c);
static int comm_abort(g2v_ctx* c, const char* why);
static void group_abort(g2v_local_group* g, const char* why);

extern "C" {

int g2v_plan_jobs(const int64_t* sent_off, int64_t n_sent, int64_t sent_len, int64_t batch_words,
                  int64_t* job_sent, int64_t cap, int64_t* n_jobs_out) {
  REQUIRE(n_jobs_out != nullptr, G2V_EINVAL, "n_jobs_out is null");
  REQUIRE(n_sent >= 0 && batch_words > 0, G2V_EINVAL, "bad sizes");
  REQUIRE(sent_len > 0 || sent_off, G2V_EINVAL, "need sent_off or sent_len > 0");
  // [ext] _job_producer: `if batch_size + len <= batch_words: append else: push`
  if (sent_len > 0) {
    // fixed-length sentences: the loop below packs exactly
    // floor(batch_words / sent_len) sentences per job, so the starts are a
    // closed form (no O(n_sent) pass per train() call: 100 M pairs cost 73 ms)
    if (sent_len > batch_words && n_sent > 0) {
      // every sentence overflows a job: the producer first queues the empty
      // job, then each sentence alone -> {0, 0, 1, ..., n_sent}
      const int64_t nj = n_sent + 1;
      if (job_sent)
        for (int64_t j = 0; j <= nj && j < cap; ++j) job_sent[j] = j == 0 ? 0 : j - 1;
      *n_jobs_out = nj;
      if (job_sent && cap < nj + 1)
        return fail(G2V_ERANGE, "job_sent capacity %lld < %lld", (long long)cap,
                    (long long)(nj + 1));
      return G2V_OK;
    }
    const int64_t per = n_sent ? batch_words / sent_len : 1;
    const int64_t nj = (n_sent + per - 1) / per;
    if (job_sent)
      for (int64_t j = 0; j <= nj && j < cap; ++j) job_sent[j] = j < nj ? j * per : n_sent;
    *n_jobs_out = nj;
    if (job_sent && cap < nj + 1)
      return fail(G2V_ERANGE, "job_sent capacity %lld < %lld", (long long)cap, (long long)(nj + 1));
    return G2V_OK;
  }
  int64_t nj = 0, size = 0, start = 0;
  auto emit = [&](int64_t s) {
    if (job_sent && nj < cap) job_sent[nj] = s;
    ++nj;
  };
  for (int64_t i = 0; i < n_sent; ++i) {
    const int64_t ln = sent_len > 0 ? sent_len : sent_off[i + 1] - sent_off[i];
    if (size + ln <= batch_words) {
      size += ln;
    } else {
      emit(start);
      start = i;
      size = ln;
    }
  }
  if (n_sent > start) emit(start);
  if (job_sent && nj < cap) job_sent[nj] = n_sent;
  *n_jobs_out = nj;
  if (job_sent && cap < nj + 1)
    return fail(G2V_ERANGE, "job_sent capacity %lld < %lld", (long long)cap, (long long)(nj + 1));
  return G2V_OK;
}

}  // extern "C"

static int train_impl(g2v_ctx* c, const int64_t* job_sent, const float* job_alpha,
                      const uint64_t* job_seed, int64_t n_jobs, uint32_t flags);

extern "C" {

int g2v_train(g2v_ctx* c, const int64_t* job_sent, const float* job_alpha, const uint64_t* job_seed,
              int64_t n_jobs, uint32_t flags) {
  int rc = set_dev(c);
  if (rc) return rc;
  const bool merging = c->comm_kind != kCommNone && c->merge_every > 0;
  rc = train_impl(c, job_sent, job_alpha, job_seed, n_jobs, flags);
  if (rc && merging) {
    // the peers may already wait in one of this call's merges (or will wait
    // in the next one): leave the communicator so they fail instead of hanging
    const std::string msg = g_err;
    comm_abort(c, msg.c_str());
    g_err = msg + " (communicator aborted)";
  }
  return rc;
}

}  // extern "C"

static int train_impl(g2v_ctx* c, const int64_t* job_sent, const float* job_alpha,
                      const uint64_t* job_seed, int64_t n_jobs, uint32_t flags) {
  int rc;
  REQUIRE(c->vocab_ready, G2V_ESTATE, "g2v_set_vocab must precede g2v_train");
  REQUIRE(c->corpus_ready, G2V_ESTATE, "g2v_set_corpus must precede g2v_train");
  REQUIRE(job_alpha && job_seed, G2V_EINVAL, "job_alpha / job_seed is null");
  const int mode = (int)(flags & G2V_MODE_MASK);
  REQUIRE(mode == kModeHogwild || mode == kModeSequential, G2V_EINVAL,
          "g2v_train mode must be HOGWILD or SEQUENTIAL");
  if ((rc = check_jobs(c, job_sent, n_jobs))) return rc;
  if (n_jobs == 0) return G2V_OK;
  const bool timing = flags & G2V_FLAG_TIMING;
  const bool closs = flags & G2V_FLAG_COMPUTE_LOSS;
  if ((rc = upload_jobs(c, job_sent, job_alpha, job_seed, n_jobs))) return rc;
  // segments of <= seg_jobs jobs; with G2V_OPT_MERGE_EVERY_JOBS and a
  // communicator, windows of merge_every jobs end with a replica merge
  // (g2v_average's kernels and all-reduce on the same stream), so a whole
  // data-parallel epoch is one call and the sampler overlap spans the merges
  struct Seg {
    int64_t j0, nj;
    bool merge;
    float amax;  // the segment's largest alpha (the stability cap)
  };
  std::vector<Seg> segs;
  const bool merging = c->comm_kind != kCommNone && c->merge_every > 0;
  const int64_t win = merging ? c->merge_every : n_jobs;
  for (int64_t w0 = 0; w0 < n_jobs; w0 += win) {
    const int64_t w1 = std::min<int64_t>(n_jobs, w0 + win);
    for (int64_t j0 = w0; j0 < w1; j0 += c->seg_jobs) {
      const int64_t nj = std::min<int64_t>(c->seg_jobs, w1 - j0);
      float am = 0.f;
      if (mode == kModeHogwild)
        for (int64_t j = j0; j < j0 + nj; ++j) am = std::max(am, job_alpha[j]);
      segs.push_back({j0, nj, merging && j0 + nj == w1, am});
    }
  }
  const int64_t n_seg = (int64_t)segs.size();
  int64_t merges = 0;
  auto merge = [&]() -> int {
    if (++merges == c->debug_fail_merge)
      return fail(G2V_ECOMM, "injected failure before in-call merge %lld (G2V_OPT_DEBUG_FAIL_MERGE)",
                  (long long)merges);
    return merge_now(c, c->merge_rule);
  };
  if (!c->sample_overlap || n_seg == 1) {
    for (const Seg& g : segs) {
      if ((rc = sample_segment(c, g.j0, g.nj, timing))) return rc;
      if ((rc = run_sgns(c, c->d_job_exoff + g.nj, mode, timing, closs, c->syn0, c->syn1,
                         nullptr, g.amax)))
        return rc;
      if (g.merge && (rc = merge())) return rc;
    }
    c->jobs += n_jobs;
    return G2V_OK;
  }
  // two-stage pipeline over double-buffered segment workspaces: segment s+1 is
  // sampled on the side stream under segment s's SGNS kernel; the segments
  // still train in order on the context's stream
  if (!c->side) {
    HIPCHK(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
    for (hipEvent_t* e : {&c->ev_up, &c->ev_samp[0], &c->ev_samp[1], &c->ev_sgns[0],
                          &c->ev_sgns[1]})
      HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  HIPCHK(hipEventRecord(c->ev_up, c->stream));  // job tables uploaded, counters reset
  HIPCHK(hipStreamWaitEvent(c->side, c->ev_up, 0));
  if ((rc = sample_segment(c, segs[0].j0, segs[0].nj, timing, 0, c->side))) return rc;
  HIPCHK(hipEventRecord(c->ev_samp[0], c->side));
  for (int64_t sg = 0; sg < n_seg; ++sg) {
    const int b = (int)(sg & 1);
    const Seg& g = segs[(size_t)sg];
    if (sg + 1 < n_seg) {
      const Seg& h = segs[(size_t)sg + 1];
      // workspace 1-b was last read by segment sg-1's SGNS kernel
      if (sg >= 1) HIPCHK(hipStreamWaitEvent(c->side, c->ev_sgns[1 - b], 0));
      if ((rc = sample_segment(c, h.j0, h.nj, timing, 1 - b, c->side))) return rc;
      HIPCHK(hipEventRecord(c->ev_samp[1 - b], c->side));
    }
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_samp[b], 0));
    if ((rc = run_sgns(c, (b ? c->d_job_exoff2 : c->d_job_exoff) + g.nj, mode, timing, closs,
                       c->syn0, c->syn1, b ? c->d_rec2 : c->d_rec, g.amax)))
      return rc;
    HIPCHK(hipEventRecord(c->ev_sgns[b], c->stream));
    if (g.merge && (rc = merge())) return rc;
  }
  c->jobs += n_jobs;
  return G2V_OK;
}

extern "C" {

int g2v_debug_sample(g2v_ctx* c, const int64_t* job_sent, const uint64_t* job_seed, int64_t n_jobs,
                     int32_t* rec_out, int64_t cap, int64_t* n_out) {
  int rc = set_dev(c);
  if (rc) return rc;
  REQUIRE(c->vocab_ready && c->corpus_ready, G2V_ESTATE, "vocab and corpus required");
  REQUIRE(n_out != nullptr && job_seed != nullptr, G2V_EINVAL, "null argument");
  if ((rc = check_jobs(c, job_sent, n_jobs))) return rc;
  *n_out = 0;
  if (n_jobs == 0) return G2V_OK;
  if ((rc = upload_jobs(c, job_sent, nullptr, job_seed, n_jobs))) return rc;
  int64_t total = 0;
  const int K2 = c->K + 2;
  std::vector<int32_t> tmp;
  for (int64_t j0 = 0; j0 < n_jobs; j0 += c->seg_jobs) {
    const int64_t nj = std::min<int64_t>(c->seg_jobs, n_jobs - j0);
    if ((rc = sample_segment(c, j0, nj, false))) return rc;
    int64_t ne = 0;
    HIPCHK(hipMemcpyAsync(&ne, c->d_job_exoff + nj, sizeof ne, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    tmp.resize((size_t)std::max<int64_t>(ne, 1) * c->rec_stride);
    if (ne)
      HIPCHK(hipMemcpy(tmp.data(), c->d_rec, sizeof(int32_t) * ne * c->rec_stride,
                       hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < ne; ++i) {
      if (rec_out && total + i < cap) {
        int32_t* o = rec_out + (total + i) * K2;
        const int32_t* r = tmp.data() + i * c->rec_stride;
        o[0] = r[0];
        o[1] = r[1];
        for (int d = 0; d < c->K; ++d) o[2 + d] = r[3 + d];
      }
    }
    total += ne;
  }
  *n_out = total;
  return G2V_OK;
}

int g2v_sgns_step_explicit(g2v_ctx* c, const int32_t* center, const int32_t* input,
                           const int32_t* negs, int64_t n, float alpha, uint32_t flags) {
  int rc = set_dev(c);
  if (rc) return rc;
  REQUIRE(center && input && negs, G2V_EINVAL, "null argument");
  REQUIRE(n >= 0, G2V_EINVAL, "n < 0");
  const int mode = (int)(flags & G2V_MODE_MASK);
  REQUIRE(mode <= kModeMinibatch, G2V_EINVAL, "bad mode %d", mode);
  for (int64_t i = 0; i < n; ++i) {
    REQUIRE(center[i] >= 0 && center[i] < c->V && input[i] >= 0 && input[i] < c->V, G2V_EINVAL,
            "example %lld index out of range", (long long)i);
    for (int d = 0; d < c->K; ++d)
      REQUIRE(negs[i * c->K + d] >= -1 && negs[i * c->K + d] < c->V, G2V_EINVAL,
              "example %lld negative %d out of range", (long long)i, d);
  }
  if (n == 0) return G2V_OK;
  const int64_t words = n * (2 + c->K);
  if ((rc = dev_reserve(c->stream, &c->d_ex, &c->ex_cap, words))) return rc;
  if ((rc = dev_reserve(c->stream, &c->d_rec, &c->rec_cap, n * c->rec_stride))) return rc;
  if ((rc = dev_reserve(c->stream, &c->d_job_exoff, &c->exoff_cap, 1))) return rc;
  HIPCHK(hipMemcpyAsync(c->d_ex, center, sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_ex + n, input, sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_ex + 2 * n, negs, sizeof(int32_t) * n * c->K, hipMemcpyHostToDevice,
                        c->stream));
  HIPCHK(hipMemcpyAsync(c->d_job_exoff, &n, sizeof n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(launch_explicit_records(c->d_ex, c->d_ex + n, c->d_ex + 2 * n, n, c->K, alpha,
                                 c->rec_stride, c->d_rec, c->stream));
  const float* rd0 = c->syn0;
  const float* rd1 = c->syn1;
  if (mode == kModeMinibatch) {
    const int64_t tab = (int64_t)c->V * c->ld;
    if ((rc = dev_reserve(c->stream, &c->snap0, &c->snap0_cap, tab))) return rc;
    if ((rc = dev_reserve(c->stream, &c->snap1, &c->snap1_cap, tab))) return rc;
    HIPCHK(hipMemcpyAsync(c->snap0, c->syn0, sizeof(float) * tab, hipMemcpyDeviceToDevice,
                          c->stream));
    HIPCHK(hipMemcpyAsync(c->snap1, c->syn1, sizeof(float) * tab, hipMemcpyDeviceToDevice,
                          c->stream));
    rd0 = c->snap0;
    rd1 = c->snap1;
  }
  if ((rc = run_sgns(c, c->d_job_exoff, mode, flags & G2V_FLAG_TIMING,
                     flags & G2V_FLAG_COMPUTE_LOSS, rd0, rd1)))
    return rc;
  // host arrays were copied asynchronously from pageable memory: finish before returning
  HIPCHK(hipStreamSynchronize(c->stream));
  return G2V_OK;
}

int g2v_cosine_pairs(int device, const float* vectors, int64_t V, int32_t D, const int32_t* a,
                     const int32_t* b, int64_t n, float* out) {
  REQUIRE(vectors && (n == 0 || (a && b && out)), G2V_EINVAL, "null argument");
  REQUIRE(V > 0 && D > 0 && n >= 0, G2V_EINVAL, "bad sizes");
  for (int64_t i = 0; i < n; ++i)
    REQUIRE(a[i] >= 0 && a[i] < V && b[i] >= 0 && b[i] < V, G2V_EINVAL,
            "pair %lld index out of range", (long long)i);
  HIPCHK(hipSetDevice(device));
  float *dv = nullptr, *du = nullptr, *dout = nullptr;
  int32_t* dab = nullptr;
  int rc = G2V_OK;
  const size_t tab = (size_t)V * (size_t)D;
  if ((rc = dev_alloc(&dv, tab)) || (rc = dev_alloc(&du, tab)) ||
      (rc = dev_alloc(&dab, 2 * (size_t)n)) || (rc = dev_alloc(&dout, (size_t)n))) {
    dev_free(dv); dev_free(du); dev_free(dab); dev_free(dout);
    return rc;
  }
  hipError_t e = hipMemcpy(dv, vectors, tab * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess && n) e = hipMemcpy(dab, a, n * sizeof(int32_t), hipMemcpyHostToDevice);
  if (e == hipSuccess && n) e = hipMemcpy(dab + n, b, n * sizeof(int32_t), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = launch_cosine_pairs(dv, V, D, du, dab, dab + n, n, dout, nullptr);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess && n) e = hipMemcpy(out, dout, n * sizeof(float), hipMemcpyDeviceToHost);
  dev_free(dv); dev_free(du); dev_free(dab); dev_free(dout);
  if (e != hipSuccess) return fail(G2V_EHIP, "g2v_cosine_pairs: %s", hipGetErrorString(e));
  return G2V_OK;
}

int g2v_permute_items8(int device, const void* src, void* dst, int64_t n_items, int64_t first,
                       int64_t count, uint64_t seed, void* stream) {
  REQUIRE(n_items >= 0 && first >= 0 && count >= 0 && first <= n_items &&
              count <= n_items - first,
          G2V_EINVAL, "positions [%lld, %lld) outside the %lld items", (long long)first,
          (long long)(first + count), (long long)n_items);
  REQUIRE(count == 0 || (src && dst), G2V_EINVAL, "null device pointer");
  REQUIRE(n_items < (1ll << 62), G2V_ERANGE, "%lld items: at most 2^62", (long long)n_items);
  if (count == 0) return G2V_OK;
  HIPCHK(hipSetDevice(device));
  const PermKey pk = perm_key((uint64_t)n_items, seed);
  HIPCHK(launch_permute8(static_cast<const uint64_t*>(src), static_cast<uint64_t*>(dst), pk, first,
                         count, static_cast<hipStream_t>(stream)));
  return G2V_OK;
}

int g2v_first_occurrence_perm8(int device, const void* items, int64_t n_items, uint64_t seed,
                               int32_t n_ids, int64_t* first, void* stream) {
  REQUIRE(n_items >= 0 && n_ids >= 0, G2V_EINVAL, "bad sizes");
  REQUIRE(n_items < (1ll << 62), G2V_ERANGE, "%lld items: at most 2^62", (long long)n_items);
  REQUIRE((n_items == 0 || items) && (n_ids == 0 || first), G2V_EINVAL, "null device pointer");
  if (n_ids == 0) return G2V_OK;
  HIPCHK(hipSetDevice(device));
  const PermKey pk = perm_key((uint64_t)n_items, seed);
  HIPCHK(launch_first_occ_perm8(static_cast<const uint64_t*>(items), pk, n_ids, first,
                                static_cast<hipStream_t>(stream)));
  return G2V_OK;
}

int g2v_sync(g2v_ctx* c) {
  int rc = set_dev(c);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(c->stream));
  return check_fault(c);
}

int g2v_debug_stamps(g2v_ctx* c, uint64_t* out, int64_t n) {
  int rc = set_dev(c);
  if (rc) return rc;
  REQUIRE(out != nullptr && n >= kStampWords, G2V_EINVAL, "need %d output words", kStampWords);
  HIPCHK(hipStreamSynchronize(c->stream));
  memset(out, 0, sizeof(uint64_t) * (size_t)n);
  if (!c->d_stamps) return G2V_OK;
  HIPCHK(hipMemcpy(out, c->d_stamps, kStampWords * sizeof(uint64_t), hipMemcpyDeviceToHost));
  HIPCHK(hipMemset(c->d_stamps, 0, kStampWords * sizeof(unsigned long long)));
  return G2V_OK;
}

int g2v_reset_loss(g2v_ctx* c) {
  int rc = set_dev(c);
  if (rc) return rc;
  HIPCHK(hipMemsetAsync(c->d_loss, 0, 2 * sizeof(double), c->stream));
  return G2V_OK;
}

int g2v_read_stats(g2v_ctx* c, g2v_stats* out) {
  int rc = set_dev(c);
  if (rc) return rc;
  REQUIRE(out != nullptr, G2V_EINVAL, "out is null");
  HIPCHK(hipStreamSynchronize(c->stream));
  if ((rc = check_fault(c))) return rc;
  unsigned long long cnt[4] = {0, 0, 0, 0};
  double loss[2] = {0.0, 0.0};
  HIPCHK(hipMemcpy(cnt, c->d_counters, sizeof cnt, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(loss, c->d_loss, sizeof loss, hipMemcpyDeviceToHost));
  HIPCHK(hipMemsetAsync(c->d_counters, 0, sizeof cnt, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  memset(out, 0, sizeof *out);
  float lf32;
  memcpy(&lf32, &loss[1], sizeof lf32);
  out->training_loss = loss[0] + (double)lf32;
  out->effective_words = (int64_t)cnt[0];
  out->examples = (int64_t)cnt[1];
  out->raw_words = (int64_t)cnt[2];
  out->jobs = c->jobs;
  out->launches = c->launches;
  out->sgns_grid = c->last_grid;
  out->stripe_rows = c->last_stripe_rows;
  out->stripe_copies = c->last_stripe_copies;
  out->stripe2_rows = c->last_stripe2_rows;
  out->stripe2_copies = c->last_stripe2_copies;
  int waves = 0;
  if (c->last_grid > 0) HIPCHK(hipMemcpy(&waves, c->d_waves, sizeof waves, hipMemcpyDeviceToHost));
  out->sgns_waves = waves;
  out->tail_row_syn0 = c->last_tail0;
  out->tail_row_syn1neg = c->last_tail1;
  for (auto& p : c->t_sgns) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, p.first, p.second));
    out->sgns_kernel_ms += ms;
  }
  for (auto& p : c->t_samp) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, p.first, p.second));
    out->sample_kernel_ms += ms;
  }
  c->t_sgns.clear();
  c->t_samp.clear();
  c->ev_used = 0;
  c->jobs = 0;
  c->launches = 0;
  return G2V_OK;
}

// ---------------------------------------------------------------------------
// multi-GPU replica averaging
// ---------------------------------------------------------------------------
int g2v_comm_unique_id(void* id_out, int64_t id_bytes) {
  REQUIRE(id_out != nullptr && id_bytes >= (int64_t)sizeof(ncclUniqueId), G2V_EINVAL,
          "id buffer must hold %zu bytes", sizeof(ncclUniqueId));
  const Rccl& r = rccl();
  REQUIRE(r.get_unique_id != nullptr, G2V_ECOMM, "RCCL unavailable: %s", r.load_error.c_str());
  ncclUniqueId id;
  NCCLCHK(r.get_unique_id(&id), "ncclGetUniqueId");
  memcpy(id_out, &id, sizeof id);
  return G2V_OK;
}

int g2v_merge_snapshot(g2v_ctx* c) {
  int rc = set_dev(c);
  if (rc) return rc;
  REQUIRE(c->weights_ready, G2V_ESTATE, "tables must be set or bound before a merge snapshot");
  const size_t tab = (size_t)c->V * (size_t)c->ld;
  if (!c->merge0 || c->merge_ld != c->ld) {
    HIPCHK(hipStreamSynchronize(c->stream));
    dev_free(c->merge0);
    dev_free(c->merge1);
    dev_free(c->merge_cnt);
    if ((rc = dev_alloc(&c->merge0, tab)) || (rc = dev_alloc(&c->merge1, tab)) ||
        (rc = dev_alloc(&c->merge_cnt, 4 * (size_t)c->V)))  // [cnt0, cnt1, nsq0, nsq1]
      return rc;
    c->merge_ld = c->ld;
  }
  HIPCHK(hipMemcpyAsync(c->merge0, c->syn0, tab * sizeof(float), hipMemcpyDeviceToDevice,
                        c->stream));
  HIPCHK(hipMemcpyAsync(c->merge1, c->syn1, tab * sizeof(float), hipMemcpyDeviceToDevice,
                        c->stream));
  c->merge_valid = true;
  return G2V_OK;
}

int g2v_comm_init(g2v_ctx* c, const void* id, int nranks, int rank) {
  int rc = set_dev(c);
  if (rc) return rc;
  REQUIRE(id != nullptr, G2V_EINVAL, "rccl_unique_id is null");
  REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, G2V_EINVAL, "rank %d of %d invalid", rank,
          nranks);
  REQUIRE(c->weights_ready, G2V_ESTATE, "set or bind the tables before g2v_comm_init");
  const Rccl& r = rccl();
  REQUIRE(r.comm_init_rank != nullptr, G2V_ECOMM, "RCCL unavailable: %s", r.load_error.c_str());
  comm_destroy(c);
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof uid);
  ncclComm_t comm = nullptr;
  NCCLCHK(r.comm_init_rank(&comm, nranks, uid, rank), "ncclCommInitRank");
  c->comm = comm;
  c->comm_kind = kCommRccl;
  c->nranks = nranks;
  c->rank = rank;
  if ((rc = comm_broadcast_tables(c))) return rc;
  return g2v_merge_snapshot(c);
}

int g2v_local_group_create(int nranks, int timeout_s, g2v_local_group** out) {
  REQUIRE(out != nullptr, G2V_EINVAL, "out is null");
  *out = nullptr;
  REQUIRE(nranks >= 1 && nranks <= kMaxLocalReplicas, G2V_EINVAL, "nranks %d out of [1, %d]",
          nranks, kMaxLocalReplicas);
  REQUIRE(timeout_s >= 0, G2V_EINVAL, "timeout_s < 0");
  g2v_local_group* g = new (std::nothrow) g2v_local_group();
  REQUIRE(g != nullptr, G2V_ENOMEM, "group allocation failed");
  g->n = nranks;
  g->timeout_s = timeout_s ? timeout_s : 600;
  g->joined.assign((size_t)nranks, 0);
  g->ev.assign((size_t)nranks, nullptr);
  g->bufs.assign((size_t)nranks, {nullptr, nullptr, nullptr});
  *out = g;
  return G2V_OK;
}

int g2v_local_group_destroy(g2v_local_group* g) {
  if (!g) return G2V_OK;
  if (g->device >= 0) (void)hipSetDevice(g->device);
  (void)hipDeviceSynchronize();
  for (hipEvent_t e : g->ev)
    if (e) (void)hipEventDestroy(e);
  if (g->ev_done) (void)hipEventDestroy(g->ev_done);
  dev_free(g->scratch);
  delete g;
  return G2V_OK;
}

int g2v_comm_init_local(g2v_ctx* c, g2v_local_group* g, int rank) {
  int rc = set_dev(c);
  if (rc) return rc;
  REQUIRE(g != nullptr, G2V_EINVAL, "group is null");
  REQUIRE(rank >= 0 && rank < g->n, G2V_EINVAL, "rank %d of %d invalid", rank, g->n);
  REQUIRE(c->weights_ready, G2V_ESTATE, "set or bind the tables before g2v_comm_init_local");
  {
    std::lock_guard<std::mutex> lk(g->mu);
    if (g->device < 0) {
      g->device = c->device;
      g->V = c->V;
      g->ld = c->ld;
    }
    if (g->device != c->device || g->V != c->V || g->ld != c->ld) {
      g->aborted = true;
      g->why = "ranks differ in device / V / ld";
      g->cv.notify_all();
      return fail(G2V_EINVAL, "rank %d: device / V / ld differ from the group's", rank);
    }
    // every failure from here on aborts the group (under its lock), so the
    // ranks already waiting in local_broadcast's barrier fail at once
    auto abort_locked = [&](int code) {
      g->aborted = true;
      g->why = g_err;
      g->cv.notify_all();
      return code;
    };
    if (g->joined[(size_t)rank])
      return abort_locked(fail(G2V_EINVAL, "rank %d joined twice", rank));
    g->joined[(size_t)rank] = 1;
    hipError_t he = hipSuccess;
    if (!g->ev[(size_t)rank] &&
        (he = hipEventCreateWithFlags(&g->ev[(size_t)rank], hipEventDisableTiming)) != hipSuccess)
      return abort_locked(fail(G2V_EHIP, "hipEventCreate failed: %s", hipGetErrorString(he)));
    if (rank == 0) {
      if ((he = hipEventCreateWithFlags(&g->ev_done, hipEventDisableTiming)) != hipSuccess)
        return abort_locked(fail(G2V_EHIP, "hipEventCreate failed: %s", hipGetErrorString(he)));
      // both tables and both touched-count vectors of one merge
      const size_t need = 2 * (size_t)c->V * (size_t)c->ld + 4 * (size_t)c->V;
      if ((rc = dev_alloc(&g->scratch, need))) return abort_locked(rc);
      g->scratch_cap = need;
    }
  }
  comm_destroy(c);
  c->lgroup = g;
  c->comm_kind = kCommLocal;
  c->nranks = g->n;
  c->rank = rank;
  if ((rc = comm_broadcast_tables(c))) return rc;
  return g2v_merge_snapshot(c);
}

int g2v_comm_init_host(g2v_ctx* c, g2v_collective_fn fn, void* user, int nranks, int rank) {
  int rc = set_dev(c);
  if (rc) return rc;
  REQUIRE(fn != nullptr, G2V_EINVAL, "collective callback is null");
  REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, G2V_EINVAL, "rank %d of %d invalid", rank,
          nranks);
  REQUIRE(c->weights_ready, G2V_ESTATE, "set or bind the tables before g2v_comm_init_host");
  comm_destroy(c);
  c->host_fn = fn;
  c->host_user = user;
  c->comm_kind = kCommHost;
  c->nranks = nranks;
  c->rank = rank;
  if ((rc = comm_broadcast_tables(c))) return rc;
  return g2v_merge_snapshot(c);
}

int g2v_comm_abort(g2v_ctx* c) {
  int rc = set_dev(c);
  if (rc) return rc;
  return comm_abort(c, "g2v_comm_abort");
}

int g2v_average(g2v_ctx* c, int rule) {
  int rc = set_dev(c);
  if (rc) return rc;
  REQUIRE(rule == G2V_MERGE_TOUCH || rule == G2V_MERGE_MEAN || rule == G2V_MERGE_ALIGN, G2V_EINVAL,
          "merge rule %d", rule);
  if (c->comm_kind == kCommNone) return G2V_OK;  // no communicator: nothing to merge with
  rc = merge_now(c, rule);
  if (rc) {
    const std::string msg = g_err;
    comm_abort(c, msg.c_str());
    g_err = msg + " (communicator aborted)";
  }
  return rc;
}

}  // extern "C"

// ---- transports -------------------------------------------------------------------
// a failing rank aborts the in-process group so its peers do not wait forever
#define GCHK(x)                                       \
  do {                                                \
    const int rc_ = (x);                              \
    if (rc_) {                                        \
      group_abort(g, g_err.c_str());                  \
      return rc_;                                     \
    }                                                 \
  } while (0)
#define GHIP(x)                                                                      \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      const int rc_ = fail(G2V_EHIP, "%s failed: %s", #x, hipGetErrorString(e_));    \
      group_abort(g, g_err.c_str());                                                 \
      return rc_;                                                                    \
    }                                                                                \
  } while (0)

static void group_abort(g2v_local_group* g, const char* why) {
  std::lock_guard<std::mutex> lk(g->mu);
  if (!g->aborted) {
    g->aborted = true;
    g->why = why ? why : "?";
  }
  g->cv.notify_all();
}

// host barrier of the group's ranks (a collective's meeting point)
static int group_wait(g2v_local_group* g) {
  std::unique_lock<std::mutex> lk(g->mu);
  if (g->aborted) return fail(G2V_ECOMM, "replica group aborted: %s", g->why.c_str());
  const uint64_t my = g->gen;
  if (++g->arrived == g->n) {
    g->arrived = 0;
    ++g->gen;
    g->cv.notify_all();
    return G2V_OK;
  }
  const bool done = g->cv.wait_for(lk, std::chrono::seconds(g->timeout_s),
                                   [&] { return g->gen != my || g->aborted; });
  if (g->gen != my) return G2V_OK;
  if (!done && !g->aborted) {
    g->aborted = true;
    g->why = "a rank did not reach the barrier within the timeout";
    g->cv.notify_all();
  }
  return fail(G2V_ECOMM, "replica group aborted: %s", g->why.c_str());
}

// in place: bufs[b][0, n[b]) <- sum over the group's ranks
static int local_allreduce(g2v_ctx* c, float* const* bufs, const size_t* n, int nb) {
  g2v_local_group* g = c->lgroup;
  const int r = c->rank;
  size_t total = 0;
  for (int b = 0; b < nb; ++b) total += n[b];
  if (total > g->scratch_cap) {
    const int rc = fail(G2V_EINVAL, "collective of %zu floats exceeds the group's %zu", total,
                        g->scratch_cap);
    group_abort(g, g_err.c_str());
    return rc;
  }
  for (int b = 0; b < nb; ++b) g->bufs[(size_t)r][(size_t)b] = bufs[b];
  GHIP(hipEventRecord(g->ev[(size_t)r], c->stream));  // this rank's inputs are ready
  GCHK(group_wait(g));
  if (r == 0) {
    for (int q = 0; q < g->n; ++q) GHIP(hipStreamWaitEvent(c->stream, g->ev[(size_t)q], 0));
    size_t off = 0;
    for (int b = 0; b < nb; ++b) {
      SumArgs sa{};
      for (int q = 0; q < g->n; ++q) sa.src[q] = g->bufs[(size_t)q][(size_t)b];
      GHIP(launch_sum_replicas(sa, g->n, g->scratch + off, (int64_t)n[b], c->stream));
      off += n[b];
    }
    GHIP(hipEventRecord(g->ev_done, c->stream));
  }
  GCHK(group_wait(g));
  // the next collective's sum waits for these copies (it waits for every
  // rank's next ready event, recorded after them on the rank's stream)
  if (r != 0) GHIP(hipStreamWaitEvent(c->stream, g->ev_done, 0));
  size_t off = 0;
  for (int b = 0; b < nb; ++b) {
    GHIP(hipMemcpyAsync(bufs[b], g->scratch + off, n[b] * sizeof(float), hipMemcpyDeviceToDevice,
                        c->stream));
    off += n[b];
  }
  return G2V_OK;
}

// in place: bufs[b] <- rank 0's bufs[b]
static int local_broadcast(g2v_ctx* c, float* const* bufs, const size_t* n, int nb) {
  g2v_local_group* g = c->lgroup;
  const int r = c->rank;
  for (int b = 0; b < nb; ++b) g->bufs[(size_t)r][(size_t)b] = bufs[b];
  GHIP(hipEventRecord(g->ev[(size_t)r], c->stream));
  GCHK(group_wait(g));
  if (r != 0) {
    GHIP(hipStreamWaitEvent(c->stream, g->ev[0], 0));
    for (int b = 0; b < nb; ++b)
      GHIP(hipMemcpyAsync(bufs[b], g->bufs[0][(size_t)b], n[b] * sizeof(float),
                          hipMemcpyDeviceToDevice, c->stream));
    GHIP(hipEventRecord(g->ev[(size_t)r], c->stream));
  }
  GCHK(group_wait(g));
  // rank 0's tables change again only after every copy of them was taken
  if (r == 0)
    for (int q = 1; q < g->n; ++q) GHIP(hipStreamWaitEvent(c->stream, g->ev[(size_t)q], 0));
  return G2V_OK;
}

// host transport: device -> pinned host, the caller's collective, back
static int host_collective(g2v_ctx* c, int op, float* const* bufs, const size_t* n, int nb) {
  size_t total = 0;
  for (int b = 0; b < nb; ++b) total += n[b];
  if (total > c->h_coll_cap) {
    if (c->h_coll) HIPCHK(hipHostFree(c->h_coll));
    c->h_coll = nullptr;
    c->h_coll_cap = 0;
    HIPCHK(hipHostMalloc((void**)&c->h_coll, total * sizeof(float), hipHostMallocDefault));
    c->h_coll_cap = total;
  }
  size_t off = 0;
  for (int b = 0; b < nb; ++b) {
    HIPCHK(hipMemcpyAsync(c->h_coll + off, bufs[b], n[b] * sizeof(float), hipMemcpyDeviceToHost,
                          c->stream));
    off += n[b];
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  const int e = c->host_fn(c->host_user, op, c->h_coll, (int64_t)total);
  REQUIRE(e == 0, G2V_ECOMM, "host collective callback (op %d, %zu floats) returned %d", op, total,
          e);
  off = 0;
  for (int b = 0; b < nb; ++b) {
    HIPCHK(hipMemcpyAsync(bufs[b], c->h_coll + off, n[b] * sizeof(float), hipMemcpyHostToDevice,
                          c->stream));
    off += n[b];
  }
  HIPCHK(hipStreamSynchronize(c->stream));  // the staging is reused by the next collective
  return G2V_OK;
}

// every replica starts from rank 0's tables (Python's hash() seeds the
// reference's init differently in every process)
static int comm_broadcast_tables(g2v_ctx* c) {
  if (c->nranks <= 1) return G2V_OK;
  const size_t tab = (size_t)c->V * (size_t)c->ld;
  float* bufs[2] = {c->syn0, c->syn1};
  const size_t n[2] = {tab, tab};
  switch (c->comm_kind) {
    case kCommRccl: {
      const Rccl& r = rccl();
      NCCLCHK(r.group_start(), "ncclGroupStart");
      for (int k = 0; k < 2; ++k)
        NCCLCHK(r.broadcast(bufs[k], bufs[k], tab, ncclFloat32, 0, c->comm, c->stream),
                "ncclBroadcast");
      NCCLCHK(r.group_end(), "ncclGroupEnd");
      return G2V_OK;
    }
    case kCommLocal: return local_broadcast(c, bufs, n, 2);
    case kCommHost: return host_collective(c, G2V_COLL_BCAST0, bufs, n, 2);
    default: return fail(G2V_ESTATE, "no communicator");
  }
}

// in place: bufs[b] <- sum over ranks (one grouped collective)
static int comm_allreduce(g2v_ctx* c, float* const* bufs, const size_t* n, int nb) {
  switch (c->comm_kind) {
    case kCommRccl: {
      const Rccl& r = rccl();
      NCCLCHK(r.group_start(), "ncclGroupStart");
      for (int b = 0; b < nb; ++b)
        NCCLCHK(r.all_reduce(bufs[b], bufs[b], n[b], ncclFloat32, ncclSum, c->comm, c->stream),
                "ncclAllReduce");
      NCCLCHK(r.group_end(), "ncclGroupEnd");
      return G2V_OK;
    }
    case kCommLocal: return local_allreduce(c, bufs, n, nb);
    case kCommHost: return host_collective(c, G2V_COLL_SUM, bufs, n, nb);
    default: return fail(G2V_ESTATE, "no communicator");
  }
}

static int comm_abort(g2v_ctx* c, const char* why) {
  if (c->comm_kind == kCommRccl && c->comm) {
    const Rccl& r = rccl();
    if (r.comm_abort) (void)r.comm_abort(c->comm);
    else if (r.comm_destroy) (void)r.comm_destroy(c->comm);
    c->comm = nullptr;
  } else if (c->comm_kind == kCommLocal && c->lgroup) {
    group_abort(c->lgroup, why);
  }
  c->comm_kind = kCommNone;
  c->lgroup = nullptr;
  c->host_fn = nullptr;
  c->host_user = nullptr;
  c->nranks = 1;
  c->rank = 0;
  return G2V_OK;
}

// the merge of g2v_average on the context's stream (also run inside g2v_train
// at G2V_OPT_MERGE_EVERY_JOBS window ends); a one-rank communicator runs the
// full path, an identity on the values
static int merge_now(g2v_ctx* c, int rule) {
  REQUIRE(c->merge_valid && c->merge_ld == c->ld, G2V_ESTATE,
          "no merge snapshot (g2v_comm_init* / g2v_merge_snapshot)");
  const size_t tab = (size_t)c->V * (size_t)c->ld;
  float* t[2] = {c->syn0, c->syn1};
  float* o[2] = {c->merge0, c->merge1};
  float* cnt = c->merge_cnt;                 // [2][V] touched flags, then counts
  float* nsq = c->merge_cnt + 2 * (size_t)c->V;  // [2][V] squared delta norms, then sums
  if (rule != G2V_MERGE_MEAN)
    for (int k = 0; k < 2; ++k)
      HIPCHK(launch_merge_delta(t[k], o[k], cnt + (size_t)k * c->V, nsq + (size_t)k * c->V, c->V,
                                c->ld, c->nvec, c->stream));
  // one grouped collective: both tables, then the counts (and norms)
  float* bufs[3] = {t[0], t[1], cnt};
  const size_t n[3] = {tab, tab, (rule == G2V_MERGE_ALIGN ? 4 : 2) * (size_t)c->V};
  int rc = comm_allreduce(c, bufs, n, rule == G2V_MERGE_MEAN ? 2 : 3);
  if (rc) return rc;
  for (int k = 0; k < 2; ++k)
    HIPCHK(launch_merge_apply(t[k], o[k], cnt + (size_t)k * c->V, nsq + (size_t)k * c->V, c->V,
                              c->ld, c->nvec, rule, 1.0f / (float)c->nranks, c->merge_beta,
                              c->merge_gamma, c->stream));
  return G2V_OK;
}

extern "C" {

int g2v_average_local(g2v_ctx* const* ctxs, int n, int rule) {
  REQUIRE(ctxs != nullptr && n >= 1 && n <= kMaxLocalReplicas, G2V_EINVAL,
          "need 1..%d contexts", kMaxLocalReplicas);
  REQUIRE(rule == G2V_MERGE_TOUCH || rule == G2V_MERGE_MEAN || rule == G2V_MERGE_ALIGN, G2V_EINVAL,
          "merge rule %d", rule);
  g2v_ctx* c0 = ctxs[0];
  int rc = set_dev(c0);
  if (rc) return rc;
  LocalMergeArgs a{};
  for (int i = 0; i < n; ++i) {
    g2v_ctx* c = ctxs[i];
    REQUIRE(c != nullptr, G2V_EINVAL, "context %d is null", i);
    REQUIRE(c->device == c0->device && c->V == c0->V && c->D == c0->D && c->ld == c0->ld,
            G2V_EINVAL, "context %d differs in device / V / D / ld", i);
    REQUIRE(c->merge_valid && c->merge_ld == c->ld, G2V_ESTATE,
            "context %d has no merge snapshot (g2v_merge_snapshot)", i);
    // the merge reads every replica: their queued work must be done
    if (c->stream != c0->stream) HIPCHK(hipStreamSynchronize(c->stream));
  }
  for (int k = 0; k < 2; ++k) {
    for (int i = 0; i < n; ++i) {
      a.t[i] = k ? ctxs[i]->syn1 : ctxs[i]->syn0;
      a.old[i] = k ? ctxs[i]->merge1 : ctxs[i]->merge0;
    }
    HIPCHK(launch_merge_local(a, n, c0->V, c0->ld, c0->nvec, rule, c0->merge_beta, c0->merge_gamma,
                              c0->stream));
  }
  // later work on the other contexts' streams must see the merged tables
  bool other = false;
  for (int i = 1; i < n; ++i) other |= ctxs[i]->stream != c0->stream;
  if (other) HIPCHK(hipStreamSynchronize(c0->stream));
  return G2V_OK;
}

}  // extern "C"
