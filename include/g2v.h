/*
 * g2v.h -- C ABI of libg2v.so, the MI355X-native Gene2vec SGNS engine.
 *
 * The reference's hot path is gensim 3.4.0's skip-gram negative-sampling
 * trainer driven from src/gene2vec.py.  Its plug-in point is gensim's per-job
 * hook [ext] Word2Vec._do_train_job(sentences, alpha, inits) ->
 * word2vec_inner.train_batch_sg(model, sentences, alpha, work, compute_loss),
 * called from BaseAny2VecModel._worker_loop threads; the whole hook sits behind
 * the Python API used at src/gene2vec.py:70 (Word2Vec(...)), :86 (load) and
 * :87 (model.train(...)).  gensim reaches it through Cython, not a C FFI; this
 * header is the C ABI a ctypes binding (gene2vec_amd/_native.py) loads in its
 * place.  Every entry point below cites the reference behaviour it replaces
 * ([ext] = upstream gensim 3.4.0).
 *
 * Conventions
 *   - C linkage, POD arguments only, no torch types.
 *   - Every function returns int status: G2V_OK (0) or a negative G2V_E* code;
 *     the message is in g2v_last_error() (thread-local).  Nothing aborts or
 *     throws across the ABI.
 *   - Host pointers are borrowed for the duration of the call only.  Device
 *     pointers passed to g2v_bind_tables / g2v_set_corpus(G2V_CORPUS_DEVICE)
 *     are borrowed until replaced or until g2v_destroy.
 *   - All device work is enqueued on the context's HIP stream and is
 *     asynchronous unless a function says it synchronises.
 *   - Tables live on the device as [V][ld] fp32 rows, ld = row stride in
 *     floats (a multiple of 32, i.e. 128-B aligned rows); the pad columns are
 *     kept at zero.  Host-side tables are dense [V][D] row-major fp32.
 */
#ifndef G2V_H
#define G2V_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define G2V_ABI_VERSION 5

/* status codes */
#define G2V_OK 0
#define G2V_EINVAL (-1)     /* bad argument / unsupported configuration */
#define G2V_EHIP (-2)       /* HIP runtime error */
#define G2V_ENOMEM (-3)     /* allocation failed */
#define G2V_ESTATE (-4)     /* call order violated (e.g. train before vocab) */
#define G2V_ERANGE (-5)     /* input exceeds a documented limit */
#define G2V_ECOMM (-6)      /* RCCL error or RCCL unavailable */

/* g2v_train / g2v_sgns_step_explicit modes */
#define G2V_MODE_HOGWILD 0    /* production: many waves, lock-free (gensim workers=N) */
#define G2V_MODE_SEQUENTIAL 1 /* one wave, examples in gensim order (workers=1) */
#define G2V_MODE_MINIBATCH 2  /* step API only: all examples read the pre-step tables,
                                 deltas summed (float atomics) */
#define G2V_MODE_MASK 0x3u
#define G2V_FLAG_TIMING 0x100u /* record HIP events around each SGNS kernel launch */
/* [ext] train_batch_sg(..., compute_loss=True): tally -log(sigmoid(+-f)) from
 * LOG_TABLE for every applied target into the running training loss (see
 * g2v_stats.training_loss / g2v_reset_loss).  Off: the kernels pay nothing. */
#define G2V_FLAG_COMPUTE_LOSS 0x200u

/* g2v_set_corpus flags */
#define G2V_CORPUS_DEVICE 0x1u /* tokens / sent_off are device pointers (borrowed) */

/* limits */
#define G2V_BATCH_WORDS 10000   /* gensim batch_words = MAX_SENTENCE_LEN */
#define G2V_MAX_DIM 512
#define G2V_EXP_TABLE_SIZE 1000

typedef struct g2v_ctx g2v_ctx;

typedef struct g2v_stats {
    int64_t raw_words;        /* tokens in the trained sentences (gensim raw_word_count) */
    int64_t effective_words;  /* tokens kept after OOV removal + downsampling (train_batch_sg's return) */
    int64_t examples;         /* directed (center, context) SGNS examples trained */
    int64_t jobs;             /* gensim jobs (<= 10000 raw words each) */
    int64_t launches;         /* SGNS-kernel launches */
    double sgns_kernel_ms;    /* sum of SGNS-kernel durations (G2V_FLAG_TIMING), else 0 */
    double sample_kernel_ms;  /* sum of sampling-kernel durations (G2V_FLAG_TIMING), else 0 */
    /* running training loss since the last g2v_reset_loss (NOT reset by
     * g2v_read_stats; gensim's model.running_training_loss, reset by every
     * train() call).  SEQUENTIAL launches continue one float32 running sum in
     * gensim order (train_batch_sg's REAL_t accumulator, bit for bit);
     * HOGWILD/MINIBATCH launches add per-wave float32 partial sums in double
     * (gensim's own workers>1 tally is a racy read-modify-write of that float). */
    double training_loss;
    /* layout of the last Hogwild SGNS launch (ABI 3): workgroups, hot-row
     * stripes (rows x copies) and the second tier (rows below stripe2_rows x
     * copies); the defaults are derived from the vocabulary at g2v_set_vocab */
    int64_t sgns_grid;
    int64_t stripe_rows, stripe_copies, stripe2_rows, stripe2_copies;
    /* waves that trained in that launch (ABI 4): sgns_grid x the active waves,
     * fewer where the stability cap held them back */
    int64_t sgns_waves;
    /* first syn0 / syn1neg row that launch wrote with plain stores instead of
     * float atomics (G2V_OPT_TAIL_STORE; ABI 5), -1 = none */
    int64_t tail_row_syn0, tail_row_syn1neg;
} g2v_stats;

/* ---- errors / version --------------------------------------------------- */
const char *g2v_last_error(void);
int g2v_abi_version(void);

/* ---- context ------------------------------------------------------------- */
/* Replaces gensim's Word2Vec(size=vector_size, window, negative, hs=0, sg=1)
 * model state ([ext] BaseWordEmbeddingsModel.__init__; src/gene2vec.py:70).
 * window must be 1 (src/gene2vec.py:62); negative in the compiled set
 * 1..20; 1 <= vector_size <= G2V_MAX_DIM. */
int g2v_create(int device, int32_t vocab_size, int32_t vector_size, int32_t negative,
               int32_t window, g2v_ctx **out);
int g2v_destroy(g2v_ctx *ctx);
/* Use an external HIP stream (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL restores the context's own stream.  Work already queued on the
 * previous stream completes first (synchronises when the stream changes). */
int g2v_set_stream(g2v_ctx *ctx, void *hip_stream);
/* Tuning knobs (defaults in brackets):
 *   G2V_OPT_HOT_ROWS      rows [0, n) -- the n most frequent genes -- are updated
 *                         with memory-side float atomics, the rest with plain
 *                         stores; -1 = all rows [-1]
 *   G2V_OPT_CACHE_POLICY  0 default, 1 write-through stores (sc1), 2 sc1 loads and
 *                         stores [1]
 *   G2V_OPT_SEG_JOBS      gensim jobs per sampling/update segment [1024]
 *   G2V_OPT_GRID          SGNS-kernel workgroups, 0 = the staleness-bounded
 *                         default, RECOMPUTED by every g2v_set_vocab from the
 *                         vocabulary; each Hogwild launch on it then trains
 *                         only as many waves as keep the hot syn0 rows from
 *                         overshooting (the launch's largest alpha and
 *                         |syn1neg|^2 measured on the device just before it;
 *                         DESIGN.md 5c; g2v_stats.sgns_waves); > 0 = fixed,
 *                         every wave trains, no cap [0]
 *   G2V_OPT_TABLE_MEM     context-owned table memory: 0 hipMalloc, 1 fine-grained,
 *                         2 uncached (re-allocates, zero-filled) [0]
 *   G2V_OPT_DEBUG_WRITE   measurement builds of the Hogwild kernel, negative 5
 *                         and vector_size <= 256 only: 2 = no table writes
 *                         (the write-free gather roof bench.py reports; breaks
 *                         training), 8 = the production kernel with s_memtime
 *                         stamps per loop segment (diagnostic build:
 *                         g2v_debug_stamps; its run time is not a measurement,
 *                         its segment SHARES are).  The throughput ablations
 *                         1, 3, 4, 5, 6, 7, 9 (profiles/r0*)
 *                         exist only in the -DG2V_ABLATIONS build
 *                         (gene2vec_amd.build.build(ablations=True)), with
 *                         10 = the lost-update probe of the tail stores
 *                         (g2v_debug_stamps [14] stores, [15] rows another
 *                         wave had changed before the store landed); any
 *                         mode this library does not compile, or a shape it
 *                         is not compiled for, is G2V_EINVAL [0]
 *   G2V_OPT_STRIPE_ROWS   hottest rows of each table striped over copies [4]
 *   G2V_OPT_STRIPE2_ROWS  second stripe tier: rows [STRIPE_ROWS, this) get
 *                         STRIPE2_COPIES copies each (<= STRIPE_ROWS = off);
 *                         -1 = auto: 20 when the SGNS grid fills every CU,
 *                         else off [-1]
 *   G2V_OPT_STRIPE2_COPIES copies per second-tier row: 2, 4 or 8 [4]
 *   G2V_OPT_STRIPE_COPIES copies per striped row, 1 = off, 0 = auto: 16 at
 *                         vector_size <= 256 or when the SGNS grid fills every
 *                         CU, 8 otherwise [0] (values stay
 *                         exact: readers sum the copies, each launch folds them
 *                         back; g2v_get_option reads the value in use)
 *   G2V_OPT_ATOMIC_OVERLAP Hogwild kernel: 1 = a wave's table atomics retire
 *                         behind its next example's compute, 0 = they land
 *                         before it (less staleness per wave, more waves
 *                         needed for the same rate) [1]
 *   G2V_OPT_SAMPLE_OVERLAP 1 = sample segment s+1 on a side stream while
 *                         segment s trains (double-buffered records; the
 *                         segments still train in order) [1]
 *   G2V_OPT_MERGE_EVERY_JOBS with a communicator (g2v_comm_init): g2v_train
 *                         ends every window of this many jobs -- and the
 *                         call's last, shorter one -- with the replica merge
 *                         of g2v_average, on the same stream; every rank must
 *                         make the same number of merges (0 = off) [0]
 *   G2V_OPT_MERGE_RULE    rule of those merges, G2V_MERGE_TOUCH / _MEAN / _ALIGN [TOUCH]
 *   G2V_OPT_MERGE_BETA_MILLI, G2V_OPT_MERGE_GAMMA_MILLI  divisor shape x 1000 of
 *                         the touch and align rules: new = old + sum_r d_r /
 *                         max(1, a^beta / gamma), a = the rule's count
 *                         (beta = gamma = 1: a itself; gamma > 1 scales the
 *                         step up, bounded by the sum; beta > 1 or gamma < 1
 *                         damps it; beta in [0, 4], gamma in [0.25, 16]);
 *                         used by g2v_average,
 *                         the in-call merges and g2v_average_local (the first
 *                         context's) [1000, 1000]
 *   G2V_OPT_ACTIVE_WAVES  Hogwild kernel: waves per workgroup that train, 1..4;
 *                         with G2V_OPT_GRID 1 and 1 wave the production kernel
 *                         runs its chunks in record order, a deterministic
 *                         update order (parity checks) [4]
 *   G2V_OPT_TAIL_STORE    Hogwild kernel, vector_size <= 512, any negative
 *                         count, at most 8 stored syn1neg rows per example (the
 *                         rest use atomics): cold rows (never a striped row;
 *                         syn1neg rows only in an example without a repeated
 *                         target) take plain write-through stores of their
 *                         new value instead of float atomics of the delta --
 *                         gensim's own unsynchronised read-modify-write, which
 *                         loses an update when another wave wrote the row
 *                         between this wave's read and its store.  -1 = auto:
 *                         the syn1neg rows other in-flight waves rarely touch
 *                         (waves x the row's updates per example <= 0.15,
 *                         from the vocabulary of g2v_set_vocab; none at <=
 *                         ~5,000 genes), syn0 (the exported vectors) all
 *                         atomic; off with fewer than 4 active waves (the
 *                         deterministic parity mode keeps its restated
 *                         all-atomic order); n > 0 = rows >= n of both
 *                         tables, 0 = off; g2v_stats reports the rows a
 *                         launch used [-1]
 *   (keys 19 and 20, G2V_OPT_ATOMIC_TAILS / G2V_OPT_COPY_DEFER of ABI 4, were
 *    retired in ABI 5: both measured slower; G2V_EINVAL)
 *   G2V_OPT_DEBUG_FAIL_MERGE fault injection (tests of the failure paths): the
 *                         n-th in-call merge of every g2v_train call fails
 *                         before its collective, as a rank that dies between
 *                         two merges would (g2v_train then leaves the
 *                         communicator); 0 = off [0] */
#define G2V_OPT_HOT_ROWS 1
#define G2V_OPT_CACHE_POLICY 2
#define G2V_OPT_SEG_JOBS 3
#define G2V_OPT_GRID 4
#define G2V_OPT_TABLE_MEM 5
#define G2V_OPT_DEBUG_WRITE 6
#define G2V_OPT_STRIPE_ROWS 7
#define G2V_OPT_STRIPE_COPIES 8
#define G2V_OPT_ATOMIC_OVERLAP 9
#define G2V_OPT_SAMPLE_OVERLAP 10
#define G2V_OPT_MERGE_EVERY_JOBS 11
#define G2V_OPT_MERGE_RULE 12
#define G2V_OPT_STRIPE2_ROWS 13
#define G2V_OPT_STRIPE2_COPIES 14
#define G2V_OPT_ACTIVE_WAVES 15
#define G2V_OPT_MERGE_BETA_MILLI 16
#define G2V_OPT_MERGE_GAMMA_MILLI 17
#define G2V_OPT_DEBUG_FAIL_MERGE 18
#define G2V_OPT_RETIRED_19 19
#define G2V_OPT_RETIRED_20 20
#define G2V_OPT_TAIL_STORE 21
int g2v_set_option(g2v_ctx *ctx, int key, int64_t value);
/* Current value of an option (G2V_OPT_GRID: the workgroups g2v_set_vocab
 * chose -- by default the staleness budget's, at most one per CU; the
 * stability cap may hold some of their waves back in a launch, and
 * g2v_read_stats reports the layout and the waves the last launch used). */
int g2v_get_option(g2v_ctx *ctx, int key, int64_t *value);
/* Row stride (floats) the device tables use. */
int g2v_row_stride(g2v_ctx *ctx, int64_t *ld_out);

/* ---- vocabulary -> sampling tables -------------------------------------- */
/* Replaces [ext] Word2VecVocab.prepare_vocab (sample_int, A.2) and
 * make_cum_table(power=ns_exponent, domain=2**31-1) (A.3).  counts are in
 * index order (sorted by descending count).  Both tables are built ON THE
 * DEVICE (sequential double accumulation, round-half-even) and are
 * bit-identical to gensim's; optional host copies are returned (synchronises
 * when either out pointer is non-NULL).  sample == 0 disables downsampling.
 * Also sizes the default Hogwild grid from the hottest row's update share. */
int g2v_set_vocab(g2v_ctx *ctx, const int64_t *counts, double sample, double ns_exponent,
                  uint32_t *cum_out, uint32_t *sample_int_out);

/* ---- weights --------------------------------------------------------------- */
/* Borrow device tables (e.g. torch-owned, so torch.distributed can all-reduce
 * them): syn0 = [ext] wv.vectors, syn1neg = [ext] trainables.syn1neg, both
 * [V][ld] fp32, ld >= D and a multiple of 4, each table below 2 GiB (the
 * kernels' 32-bit buffer offsets; G2V_ERANGE otherwise).  NULL, NULL returns
 * to context-owned tables. */
int g2v_bind_tables(g2v_ctx *ctx, float *syn0_dev, float *syn1neg_dev, int64_t ld);
/* Upload host [V][D] tables (+ optional vectors_lockf[V], NULL = ones).
 * Replaces the model-owned numpy arrays of [ext] reset_weights (A.4). */
int g2v_set_weights(g2v_ctx *ctx, const float *syn0, const float *syn1neg, const float *lockf);
/* Download to host [V][D]; either pointer may be NULL.  Synchronises. */
int g2v_get_weights(g2v_ctx *ctx, float *syn0, float *syn1neg);

/* ---- corpus ----------------------------------------------------------------- */
/* Sentences as CSR: tokens[n_tokens] int32 vocabulary indices (-1 = out of
 * vocabulary, skipped without drawing, as gensim's vlookup miss), sent_off[n_sent+1]
 * int64.  sent_off may be NULL when every sentence has length sent_len > 0
 * (gene pairs: sent_len = 2).  Replaces the list[list[str]] gensim receives at
 * src/gene2vec.py:70,87.  Without G2V_CORPUS_DEVICE the arrays are copied and
 * every id is checked to lie in [-1, V) (G2V_EINVAL otherwise).  A device
 * corpus is checked by the sampler as it reads it: an id outside [-1, V) is
 * skipped like an OOV token and latches a device fault that the next
 * g2v_sync / g2v_read_stats reports as G2V_EINVAL. */
int g2v_set_corpus(g2v_ctx *ctx, const int32_t *tokens, int64_t n_tokens, const int64_t *sent_off,
                   int64_t n_sent, int64_t sent_len, uint32_t flags);

/* ---- training ---------------------------------------------------------------- */
/* Job packing of [ext] BaseAny2VecModel._job_producer: a sentence joins the
 * current job while raw words <= batch_words, otherwise the current job is
 * queued and the sentence starts the next one.  A sentence longer than
 * batch_words therefore always trains as a job of its own, and when it is the
 * FIRST sentence the producer first queues an EMPTY job (which still draws its
 * two model.random seeds in train_batch_sg): job_sent = {0, 0, 1, ...}.
 * Writes job_sent[n_jobs+1] (sentence index boundaries) when job_sent != NULL
 * and cap >= n_jobs+1.  Host-only, no context. */
int g2v_plan_jobs(const int64_t *sent_off, int64_t n_sent, int64_t sent_len, int64_t batch_words,
                  int64_t *job_sent, int64_t cap, int64_t *n_jobs_out);

/* Train jobs [0, n_jobs) over the current corpus: the replacement of the
 * per-job hook train_batch_sg -> fast_sentence_sg_neg (A.5) for every job of a
 * train() epoch.  job_sent[n_jobs+1] sentence boundaries (g2v_plan_jobs),
 * job_alpha[n_jobs] the per-job learning rate of [ext] _update_job_params (A.6),
 * job_seed[n_jobs] the per-job next_random = 2**24*randint(2**24)+randint(2**24)
 * drawn from model.random.  Downsampling, the 48-bit LCG, the cum_table bisect and
 * the window-1 example order reproduce gensim exactly, including train_batch_sg's
 * truncation at MAX_SENTENCE_LEN = 10000 effective words (a job holding more
 * raw words must be a single sentence, as g2v_plan_jobs makes it; tokens after
 * the 10000th kept word draw nothing and train nothing).  mode selects the
 * update order (G2V_MODE_HOGWILD | G2V_MODE_SEQUENTIAL) | G2V_FLAG_TIMING |
 * G2V_FLAG_COMPUTE_LOSS. */
int g2v_train(g2v_ctx *ctx, const int64_t *job_sent, const float *job_alpha,
              const uint64_t *job_seed, int64_t n_jobs, uint32_t flags);

/* Deterministic step with explicit negatives: n examples (center[i] = gensim
 * word_index, input[i] = word2_index whose syn0 row is trained, negs[i*K..] with
 * -1 = skipped), one learning rate.  Modes SEQUENTIAL / HOGWILD / MINIBATCH,
 * optionally | G2V_FLAG_COMPUTE_LOSS. */
int g2v_sgns_step_explicit(g2v_ctx *ctx, const int32_t *center, const int32_t *input,
                           const int32_t *negs, int64_t n, float alpha, uint32_t flags);

/* [ext] BaseWordEmbeddingsModel.train resets model.running_training_loss to 0.0
 * at the start of every train() call; this is that reset. */
int g2v_reset_loss(g2v_ctx *ctx);

/* Debug/parity: the (center, input, negs[K]) records the device sampler
 * produces for jobs [0, n_jobs) (same arguments as g2v_train), written to
 * rec_out[cap][K+2] in gensim order; *n_out = record count.  Synchronises. */
int g2v_debug_sample(g2v_ctx *ctx, const int64_t *job_sent, const uint64_t *job_seed,
                     int64_t n_jobs, int32_t *rec_out, int64_t cap, int64_t *n_out);

/* Diagnostic (G2V_OPT_DEBUG_WRITE 8): shader-cycle sums of the stamped
 * Hogwild kernel over every wave of every launch since the previous call
 * (synchronises, then resets): out[0] waiting for the example's rows, [1]
 * compute (dots, sigmoid, gradients, LDS staging), [2] waiting for the
 * previous example's atomics to land, [3] issuing the next example's loads
 * (incl. summing striped rows' copies), [4] issuing this example's atomics,
 * [5] whole loop per wave (the rest is per-chunk work: record staging, the
 * work queue), [6] examples, [7] s_memtime ticks and [8] s_memrealtime ticks
 * (100 MHz) over the loops (clock = [7] / [8] x 100 MHz), [9] waves; within
 * [1]: [10] the dots and their cross-lane reduction, [11] the sigmoid lookups,
 * gradients and row updates; within [4]: [12] the first 4 rows' atomics;
 * within [3]: [13] the striped rows' copies (requested and summed before the
 * main rows are requested); n >= 16. */
int g2v_debug_stamps(g2v_ctx *ctx, uint64_t *out, int64_t n);

/* ---- sync / stats ------------------------------------------------------------ */
/* Synchronises the context's stream; reports (and clears) a latched device
 * fault of the sampler (corpus id outside [-1, V), or a multi-sentence job of
 * more than 10000 raw words in a device corpus) as G2V_EINVAL. */
int g2v_sync(g2v_ctx *ctx);
/* Accumulated since the previous call (synchronises, then resets; the running
 * training_loss is only reset by g2v_reset_loss).  Reports a latched device
 * fault like g2v_sync. */
int g2v_read_stats(g2v_ctx *ctx, g2v_stats *out);

/* ---- multi-GPU replica averaging (no reference equivalent:
 * gensim is one process, src/gene2vec.py:59) ----------------------------------- */
/* merge rules of g2v_average / g2v_average_local */
#define G2V_MERGE_TOUCH 0 /* row-wise: new = old + sum_r(d_r) / max(1, k^beta / gamma),
                             d_r = replica r's change since the last merge, k = replicas
                             whose row changed (G2V_OPT_MERGE_BETA/GAMMA_MILLI) */
#define G2V_MERGE_MEAN 1  /* plain model averaging: new = sum_r(t_r) / nranks */
#define G2V_MERGE_ALIGN 2 /* row-wise: new = old + sum_r(d_r) / max(1, a^beta / gamma),
                             a = clamp(|sum_r d_r|^2 / sum_r |d_r|^2, 1, k): a = k for
                             changes that agree (a row every replica drove to the same
                             point: their mean), 1 for independent ones (what one model
                             would have applied: their sum) */
/* rank 0 draws an RCCL unique id (128 bytes, ncclGetUniqueId) to hand to every
 * rank out of band (the Python driver broadcasts it over torch.distributed). */
int g2v_comm_unique_id(void *id_out, int64_t id_bytes);
/* Join the RCCL communicator of nranks processes (one GPU each, over xGMI),
 * broadcast rank 0's tables to every rank (ncclBroadcast) and record them as
 * the merge snapshot.  RCCL is loaded at run time (dlopen "librccl.so.1"):
 * G2V_ECOMM when it is absent.  Collective: every rank must call it. */
int g2v_comm_init(g2v_ctx *ctx, const void *rccl_unique_id, int nranks, int rank);
/* Merge the replicas of every rank in place (collective: every rank calls it
 * the same number of times): one fused HIP kernel forms the row deltas against
 * the snapshot and the touched-row counts, one ncclAllReduce (grouped) sums
 * them over xGMI on the context's stream, a second kernel applies the rule and
 * refreshes the snapshot.  No communicator: no-op; a one-rank communicator
 * runs the whole path (an identity on the values; callers skip it at N = 1). */
int g2v_average(g2v_ctx *ctx, int merge_rule);
/* Record the current tables as the merge snapshot (after replacing weights;
 * g2v_comm_init and g2v_set_weights do it when a communicator exists). */
int g2v_merge_snapshot(g2v_ctx *ctx);
/* The same merge over n contexts of ONE process on ONE device (replicas
 * trained by separate contexts, e.g. one per stream): no RCCL, one kernel.
 * Every context needs a snapshot (g2v_merge_snapshot) and equal V, D, ld. */
int g2v_average_local(g2v_ctx *const *ctxs, int n, int merge_rule);

/* Two more transports for the merge of g2v_average / G2V_OPT_MERGE_EVERY_JOBS.
 * Only the all-reduce (and the initial broadcast) changes; the delta and apply
 * kernels, the touch/mean rules and the in-call merges of g2v_train are the
 * RCCL path's own, so every merge line that runs under RCCL also runs here.
 *
 * In-process group: nranks contexts of one process on one device, each driven
 * by its own host thread (calls into different contexts may run concurrently).
 * The all-reduce is a device sum of the ranks' buffers in rank order (the order
 * of g2v_average_local, whose results it reproduces bit for bit), ordered by
 * HIP events, the ranks meeting at a host barrier.  A rank that fails inside a
 * collective aborts the group: the others return G2V_ECOMM instead of waiting
 * (also after timeout_s seconds at a barrier, 0 = 600).  The group must
 * outlive its contexts' collectives; destroy it after them. */
typedef struct g2v_local_group g2v_local_group;
int g2v_local_group_create(int nranks, int timeout_s, g2v_local_group **out);
int g2v_local_group_destroy(g2v_local_group *group);
/* Collective over the group's ranks (each calls it once, from its own thread):
 * rank 0's tables are copied to every rank, which records them as its merge
 * snapshot (as g2v_comm_init does). */
int g2v_comm_init_local(g2v_ctx *ctx, g2v_local_group *group, int rank);

/* Host transport: fn performs the collective on host memory, in place, over
 * whatever carries the ranks' traffic (e.g. torch.distributed gloo); it is
 * called on the thread of the g2v call, after the device buffers were copied to
 * pinned host memory, and must return 0 (anything else: G2V_ECOMM).
 *   G2V_COLL_SUM    buf[count] <- the sum over ranks of every rank's buf
 *   G2V_COLL_BCAST0 buf[count] <- rank 0's buf */
#define G2V_COLL_SUM 0
#define G2V_COLL_BCAST0 1
typedef int (*g2v_collective_fn)(void *user, int op, float *buf, int64_t count);
int g2v_comm_init_host(g2v_ctx *ctx, g2v_collective_fn fn, void *user, int nranks, int rank);

/* Leave the communicator after a failure: RCCL's ncclCommAbort (in-flight
 * collectives of this rank are torn down instead of waiting for peers that
 * will never arrive), the in-process group's abort (its other ranks return
 * G2V_ECOMM).  g2v_train calls it itself when it fails between in-call merges.
 * The context stays usable without a communicator. */
int g2v_comm_abort(g2v_ctx *ctx);

/* ---- text exporters ------------------------------------------------------------- */
/* Row text of the two exporters, every float32 printed as numpy's
 * str(np.float32(v)) (shortest round-trip digits; positional for
 * 1e-4 <= |v| < 1e16 and 0, else scientific with a >= 2-digit exponent):
 *   G2V_TXT_MATRIX  src/generateMatrix.py:18-24: word '\t' (str(v) ' ')*D '\n'
 *   G2V_TXT_W2V     [ext] save_word2vec_format(binary=False) rows:
 *                   word ' ' str(v) joined by ' ' '\n'
 * Line k prints vectors[rows[k]] (rows NULL = k) with ld floats per row and
 * the word words[word_off[k] .. word_off[k+1]).  out NULL: *written gets the
 * byte count only; otherwise G2V_ERANGE when cap is too small.  Host only. */
#define G2V_TXT_MATRIX 0
#define G2V_TXT_W2V 1
int g2v_format_rows(const float *vectors, int64_t ld, int32_t D, const int64_t *rows,
                    int64_t n_rows, const char *words, const int64_t *word_off, int32_t style,
                    char *out, int64_t cap, int64_t *written);
/* x[i] as str(np.float32(x[i])), one per line (test hook for the formatter). */
int g2v_format_f32(const float *x, int64_t n, char *out, int64_t cap, int64_t *written);

/* ---- producer side: co-expression pairs -------------------------------------- */
/* Replaces the per-study coexpr() of src/generate_gene_pairs.py:45-65:
 * corr = data.corr().abs(); (corr > threshold).values.nonzero(); row != col.
 * x: host [n_samples][n_genes] fp64 row-major (DataFrame.values; no NaN).
 * Writes the (row, col) gene-index pairs, both orders, no diagonal, in
 * nonzero() order (row-major) to pairs[n][2] when pairs != NULL and cap >= n;
 * *n_pairs always receives n (G2V_ERANGE when cap < n).  Columns with zero
 * variance never pair (pandas: NaN).  Standalone (own device buffers),
 * synchronises. */
int g2v_coexpr_pairs(int device, const double *x, int64_t n_samples, int64_t n_genes,
                     double threshold, int32_t *pairs, int64_t cap, int64_t *n_pairs);
/* Device time of the calling thread's last g2v_coexpr_pairs call, from HIP
 * events on its stream: the fused correlation+threshold kernel alone and the
 * whole call (H2D copy .. D2H of the pairs).  Zero before any call. */
int g2v_coexpr_last_timing(double *mask_ms, double *total_ms);

/* ---- consumer side ----------------------------------------------------------------- */
/* gensim wv.similarity for n index pairs (src/evaluation_target_function.py:38,49):
 * out[i] = dot(unitvec(v[a[i]]), unitvec(v[b[i]])), unitvec = v * (1/||v||) in
 * float32, dots accumulated in double and rounded to float.  vectors: host
 * [V][D] fp32.  Standalone (own device buffers), synchronises. */
int g2v_cosine_pairs(int device, const float *vectors, int64_t V, int32_t D, const int32_t *a,
                     const int32_t *b, int64_t n, float *out);

/* ---- device reshuffle of a pair corpus ------------------------------------------- */
/* The per-iteration reshuffle of src/gene2vec.py:80 (random.shuffle, unseeded
 * there) for a corpus resident in HBM: dst[i] = src[p(first + i)] for i < count,
 * where p is a keyed pseudo-random permutation of [0, n_items) (6-round Feistel
 * on 2h bits, 4^h >= n_items, splitmix64 round functions, cycle-walking; the
 * same seed gives the same p on every device, so data-parallel ranks gather
 * disjoint shards of one permutation).  Not CPython's shuffle: the reference
 * leaves its shuffles unseeded, so any uniform permutation is as faithful;
 * g2v_py_shuffle* keep the bit-exact host form.  src holds n_items 8-byte items
 * (one int32 pair each), dst count items, both device memory of `device`;
 * enqueued on `stream` (NULL: the null stream), no synchronisation. */
int g2v_permute_items8(int device, const void *src, void *dst, int64_t n_items, int64_t first,
                       int64_t count, uint64_t seed, void *stream);

/* The vocabulary scan ([ext] scan_vocab: gensim breaks count ties by first
 * occurrence) of the order g2v_permute_items8 gives with the same seed,
 * without materialising it: first[w] = the smallest token position (2i or
 * 2i+1 for the pair at permuted index i) of id w, -1 when w never occurs;
 * ids outside [0, n_ids) (OOV = -1) are skipped.  items: the n_items pairs as
 * 8-byte items, first: int64[n_ids], both device memory; enqueued on stream. */
int g2v_first_occurrence_perm8(int device, const void *items, int64_t n_items, uint64_t seed,
                               int32_t n_ids, int64_t *first, void *stream);

/* ---- host-native helpers (no device work) -------------------------------------- */
/* [ext] Word2VecTrainables.seeded_vector for every row: row i =
 * (RandomState(seeds[i]).rand(D) - 0.5) / D as float32, seeds[i] =
 * hash(word_i + str(seed)) & 0xffffffff computed by the caller.  MT19937
 * init_genrand + 53-bit random_sample, bit-identical to numpy's RandomState. */
int g2v_seeded_vectors(const uint32_t *seeds, int64_t n_rows, int32_t dim, float *out);
/* counts[V] and first-occurrence position first[V] (-1 = absent) of int ids in
 * [0, V) over ids[n]; the vocabulary scan of [ext] scan_vocab on pre-hashed ids. */
int g2v_count_ids(const int32_t *ids, int64_t n, int32_t V, int64_t *counts, int64_t *first);

/* ---- native ingest (src/gene2vec.py:36-47 and the shuffles at :52/:80) ----------- */
/* Reads files in the given order as windows-1252 text: universal newlines,
 * str.split() separators (ASCII whitespace, 0x1c-0x1f, 0xa0); every line is one
 * sentence (empty lines included).  Token ids follow global first occurrence.
 * Undefined windows-1252 bytes -> G2V_EINVAL (UnicodeDecodeError upstream). */
typedef struct g2v_corpus g2v_corpus;
int g2v_corpus_read(const char *const *paths, int n_paths, int n_threads, g2v_corpus **out);
int g2v_corpus_info(const g2v_corpus *c, int64_t *n_tokens, int64_t *n_sent, int64_t *n_words,
                    int64_t *word_bytes);
int g2v_corpus_export(const g2v_corpus *c, int32_t *tokens, int64_t *sent_off, int64_t *counts,
                      char *words, int64_t *word_off);
/* The length every sentence of the corpus has (2 for the pair generator's
 * files: sent_off is then implicit and need not be exported), -1 if ragged. */
int g2v_corpus_sent_len(const g2v_corpus *c, int64_t *len);
/* Sentences g2v_corpus_read would return for these files (lines under
 * universal newlines), from a newline count alone: lets the caller start
 * drawing src/gene2vec.py:52's shuffle of n pairs before the ingest ends. */
int g2v_count_lines(const char *const *paths, int n_paths, int n_threads, int64_t *out);
int g2v_corpus_free(g2v_corpus *c);
/* out sentence i = in sentence perm[i] (CSR gather) */
int g2v_csr_permute(const int32_t *tok, const int64_t *off, int64_t n_sent, const int64_t *perm,
                    int32_t *out_tok, int64_t *out_off);
/* all-pairs corpus (every sentence 2 tokens, offsets 2*i): out pair i = in
 * pair perm[i]; the offsets are unchanged by any permutation */
int g2v_pairs_permute(const int32_t *tok, int64_t n_pairs, const int64_t *perm, int32_t *out_tok);
/* CPython random.Random.shuffle(x) bit for bit; state624/pos = getstate()[1][:625],
 * updated in place (setstate afterwards keeps Python's generator in step). */
int g2v_py_shuffle(uint32_t *state624, uint32_t *pos, int64_t *x, int64_t n);
/* x = range(n), then g2v_py_shuffle (the permutation gene2vec.py:52,80 applies). */
int g2v_py_shuffle_range(uint32_t *state624, uint32_t *pos, int64_t *x, int64_t n);
/* the generator state g2v_py_shuffle(n) leaves, without the swaps (the draws
 * do not depend on the list): lets the CLI draw later iterations' reshuffles
 * (gene2vec.py:80) concurrently. */
int g2v_py_shuffle_skip(uint32_t *state624, uint32_t *pos, int64_t n);

#ifdef __cplusplus
}
#endif
#endif /* G2V_H */
