/*
 * C restatement of gensim 3.4.0 skip-gram negative sampling -- TEST
 * INFRASTRUCTURE ONLY (checker + timed CPU baseline; see oracle/__init__.py).
 * Parity unpinned: gensim is absent offline, the reference has no tests.
 *
 * Restates ([ext] = upstream gensim 3.4.0):
 *   orc_make_cum_table   [ext] Word2VecVocab.make_cum_table      (A.3)
 *   orc_sample_int       [ext] Word2VecVocab.prepare_vocab        (A.2)
 *   orc_exp_table        [ext] word2vec_inner.pyx init()          (A.5)
 *   orc_log_table        [ext] init(): LOG_TABLE[i] = <REAL_t>log(EXP_TABLE[i])
 *   orc_train_sequential [ext] train_batch_sg + fast_sentence_sg_neg, jobs in
 *                        order (= gensim with workers=1), driven the way
 *                        src/gene2vec.py:70,87 drives it
 *   orc_train_hogwild    the same per job, jobs spread over OpenMP threads
 *                        sharing the tables lock-free (= workers=N Hogwild,
 *                        src/gene2vec.py:59)
 *   orc_sample_records   the (center, input, negatives) stream of a job range
 *
 * Build: oracle/Makefile -> oracle/build/liboracle.so
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAX_EXP 6
#define EXP_TABLE_SIZE 1000
#define LUT_SCALE (EXP_TABLE_SIZE / MAX_EXP / 2) /* C integer division: 83 */
#define MAX_SENTENCE_LEN 10000
#define LCG_MASK 281474976710655ULL

static float g_exp_table[EXP_TABLE_SIZE];
static float g_log_table[EXP_TABLE_SIZE];
static int g_exp_ready = 0;

void orc_exp_table(float *out) {
    for (int i = 0; i < EXP_TABLE_SIZE; i++) {
        float x = ((float)i / (float)EXP_TABLE_SIZE * 2 - 1) * MAX_EXP;
        float e = (float)exp((double)x);
        out[i] = e / (e + 1);
    }
}

void orc_log_table(float *out) {
    float e[EXP_TABLE_SIZE];
    orc_exp_table(e);
    for (int i = 0; i < EXP_TABLE_SIZE; i++) out[i] = (float)log((double)e[i]);
}

static void ensure_exp(void) {
    if (!g_exp_ready) {
        orc_exp_table(g_exp_table);
        orc_log_table(g_log_table);
        g_exp_ready = 1;
    }
}

void orc_make_cum_table(const int64_t *counts, int32_t V, double power, uint32_t *out) {
    const double domain = 2147483647.0;
    double z = 0.0;
    for (int32_t i = 0; i < V; i++) z += pow((double)counts[i], power);
    double acc = 0.0;
    for (int32_t i = 0; i < V; i++) {
        acc += pow((double)counts[i], power);
        out[i] = (uint32_t)rint(acc / z * domain);
    }
}

void orc_sample_int(const int64_t *counts, int32_t V, double sample, uint64_t *out) {
    int64_t total = 0;
    for (int32_t i = 0; i < V; i++) total += counts[i];
    double thr;
    if (sample == 0.0) thr = (double)total;
    else if (sample < 1.0) thr = sample * (double)total;
    else thr = (double)(int64_t)(sample * (3 + sqrt(5.0)) / 2);
    for (int32_t i = 0; i < V; i++) {
        double v = (double)counts[i];
        double p = (sqrt(v / thr) + 1) * (thr / v);
        if (p >= 1.0) p = 1.0;
        out[i] = (uint64_t)rint(p * 4294967296.0);
    }
}

static inline uint64_t lcg(uint64_t nr) { return (nr * 25214903917ULL + 11ULL) & LCG_MASK; }

static inline int32_t bisect_left(const uint32_t *a, uint64_t x, int64_t lo, int64_t hi) {
    while (hi > lo) {
        int64_t mid = (lo + hi) >> 1;
        if (a[mid] >= x) hi = mid;
        else lo = mid + 1;
    }
    return (int32_t)lo;
}

/* dsdot: float products accumulated in double (4 partial sums, as a SIMD
 * BLAS dsdot does), cast to float.  Order differences are far below float
 * resolution of the result. */
static inline float dsdot(const float *a, const float *b, int D) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int k = 0;
    for (; k + 4 <= D; k += 4) {
        s0 += (double)a[k] * (double)b[k];
        s1 += (double)a[k + 1] * (double)b[k + 1];
        s2 += (double)a[k + 2] * (double)b[k + 2];
        s3 += (double)a[k + 3] * (double)b[k + 3];
    }
    for (; k < D; k++) s0 += (double)a[k] * (double)b[k];
    return (float)((s0 + s1) + (s2 + s3));
}

static inline void saxpy(float g, const float *x, float *y, int D) {
    for (int k = 0; k < D; k++) y[k] = fmaf(g, x[k], y[k]);
}

/* [ext] fast_sentence_sg_neg; returns the advanced LCG state.  negs != NULL:
 * explicit negatives (-1 = skipped) replace the LCG/bisect draw.  loss != NULL
 * (compute_loss): loss[0] -= LOG_TABLE[int((+-f + 6) * 83)] per applied target,
 * in float, in gensim's order; loss_exact != NULL: the same terms summed in
 * double (gensim's float running sum loses whole terms once it passes ~1e6). */
static uint64_t sg_neg(int K, const uint32_t *cum, int32_t V, float *syn0, float *syn1neg,
                       int64_t ld, int D, int32_t word_index, int32_t word2_index, float alpha,
                       float *work, uint64_t nr, const float *lockf, const int32_t *negs,
                       float *loss, double *loss_exact) {
    float *l1 = syn0 + (int64_t)word2_index * ld;
    memset(work, 0, sizeof(float) * D);
    for (int d = 0; d <= K; d++) {
        int32_t t;
        float label;
        if (d == 0) {
            t = word_index;
            label = 1.0f;
        } else {
            if (negs) {
                t = negs[d - 1];
                if (t < 0) continue;
            } else {
                t = bisect_left(cum, (nr >> 16) % cum[V - 1], 0, V);
                nr = lcg(nr);
            }
            if (t == word_index) continue;
            label = 0.0f;
        }
        float *row = syn1neg + (int64_t)t * ld;
        float f = dsdot(l1, row, D);
        if (f <= -MAX_EXP || f >= MAX_EXP) continue;
        if (loss || loss_exact) {
            const float fl = d == 0 ? f : -f;
            const float term = g_log_table[(int)((fl + MAX_EXP) * LUT_SCALE)];
            if (loss) *loss = *loss - term;
            if (loss_exact) *loss_exact -= (double)term;
        }
        f = g_exp_table[(int)((f + MAX_EXP) * LUT_SCALE)];
        float g = (label - f) * alpha;
        saxpy(g, row, work, D);
        saxpy(g, l1, row, D);
    }
    saxpy(lockf ? lockf[word2_index] : 1.0f, work, l1, D);
    return nr;
}

/* [ext] train_batch_sg for one job (window = 1).  kept[] is scratch of
 * MAX_SENTENCE_LEN ints, sidx[] of MAX_SENTENCE_LEN+1.  Returns effective words;
 * *n_ex gets the example count. */
static int64_t train_job(const int32_t *tok, const int64_t *sent_off, int64_t s0, int64_t s1,
                         float alpha, uint64_t nr, const uint32_t *sample_int, int sample_on,
                         const uint32_t *cum, int32_t V, float *syn0, float *syn1neg,
                         const float *lockf, int64_t ld, int D, int K, float *work, int32_t *kept,
                         int32_t *sidx, int64_t *n_ex, int32_t *rec_out, int64_t rec_cap,
                         int do_train, float *loss, double *loss_exact) {
    int32_t eff = 0, nsent = 0;
    sidx[0] = 0;
    for (int64_t s = s0; s < s1; s++) {
        int64_t b = sent_off[s], e = sent_off[s + 1];
        if (e == b) continue;
        for (int64_t t = b; t < e; t++) {
            int32_t w = tok[t];
            if (w < 0) continue;
            if (sample_on) {
                uint64_t r = nr >> 16;
                nr = lcg(nr);
                if ((uint64_t)sample_int[w] < r) continue;
            }
            kept[eff++] = w;
            if (eff == MAX_SENTENCE_LEN) break;
        }
        sidx[++nsent] = eff;
        if (eff == MAX_SENTENCE_LEN) break;
    }
    int64_t nex = 0;
    for (int32_t si = 0; si < nsent; si++) {
        int32_t a = sidx[si], z = sidx[si + 1];
        for (int32_t i = a; i < z; i++) {
            int32_t j0 = i - 1 < a ? a : i - 1;
            int32_t j1 = i + 2 > z ? z : i + 2;
            for (int32_t j = j0; j < j1; j++) {
                if (j == i) continue;
                if (do_train) {
                    nr = sg_neg(K, cum, V, syn0, syn1neg, ld, D, kept[i], kept[j], alpha, work,
                                nr, lockf, NULL, loss, loss_exact);
                } else if (rec_out && nex < rec_cap) {
                    int32_t *r = rec_out + nex * (K + 2);
                    r[0] = kept[i];
                    r[1] = kept[j];
                    for (int d = 0; d < K; d++) {
                        int32_t t = bisect_left(cum, (nr >> 16) % cum[V - 1], 0, V);
                        nr = lcg(nr);
                        r[2 + d] = (t == kept[i]) ? -1 : t;
                    }
                }
                nex++;
            }
        }
    }
    *n_ex = nex;
    return eff;
}

/* stats[0]=raw words, [1]=effective words, [2]=examples, [3]=jobs.  loss:
 * NULL, or gensim's float running training loss, continued in place;
 * loss_exact: NULL, or the same terms added in double */
void orc_train_sequential(const int32_t *tok, const int64_t *sent_off, const int64_t *job_sent,
                          int64_t n_jobs, const float *job_alpha, const uint64_t *job_seed,
                          const uint32_t *sample_int, int sample_on, const uint32_t *cum,
                          int32_t V, float *syn0, float *syn1neg, const float *lockf, int64_t ld,
                          int32_t D, int32_t K, int64_t *stats, float *loss,
                          double *loss_exact) {
    ensure_exp();
    float *work = (float *)malloc(sizeof(float) * D);
    int32_t *kept = (int32_t *)malloc(sizeof(int32_t) * MAX_SENTENCE_LEN);
    int32_t *sidx = (int32_t *)malloc(sizeof(int32_t) * (MAX_SENTENCE_LEN + 2));
    int64_t eff = 0, ex = 0;
    for (int64_t j = 0; j < n_jobs; j++) {
        int64_t nex = 0;
        eff += train_job(tok, sent_off, job_sent[j], job_sent[j + 1], job_alpha[j], job_seed[j],
                         sample_int, sample_on, cum, V, syn0, syn1neg, lockf, ld, D, K, work, kept,
                         sidx, &nex, NULL, 0, 1, loss, loss_exact);
        ex += nex;
    }
    if (stats) {
        stats[0] = sent_off[job_sent[n_jobs]] - sent_off[job_sent[0]];
        stats[1] = eff;
        stats[2] = ex;
        stats[3] = n_jobs;
    }
    free(work);
    free(kept);
    free(sidx);
}

void orc_train_hogwild(const int32_t *tok, const int64_t *sent_off, const int64_t *job_sent,
                       int64_t n_jobs, const float *job_alpha, const uint64_t *job_seed,
                       const uint32_t *sample_int, int sample_on, const uint32_t *cum, int32_t V,
                       float *syn0, float *syn1neg, const float *lockf, int64_t ld, int32_t D,
                       int32_t K, int nthreads, int64_t *stats) {
    ensure_exp();
    int64_t eff = 0, ex = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel reduction(+ : eff, ex)
    {
        float *work = (float *)malloc(sizeof(float) * D);
        int32_t *kept = (int32_t *)malloc(sizeof(int32_t) * MAX_SENTENCE_LEN);
        int32_t *sidx = (int32_t *)malloc(sizeof(int32_t) * (MAX_SENTENCE_LEN + 2));
#pragma omp for schedule(dynamic, 1)
        for (int64_t j = 0; j < n_jobs; j++) {
            int64_t nex = 0;
            eff += train_job(tok, sent_off, job_sent[j], job_sent[j + 1], job_alpha[j],
                             job_seed[j], sample_int, sample_on, cum, V, syn0, syn1neg, lockf, ld,
                             D, K, work, kept, sidx, &nex, NULL, 0, 1, NULL, NULL);
            ex += nex;
        }
        free(work);
        free(kept);
        free(sidx);
    }
    if (stats) {
        stats[0] = sent_off[job_sent[n_jobs]] - sent_off[job_sent[0]];
        stats[1] = eff;
        stats[2] = ex;
        stats[3] = n_jobs;
    }
}

/* records [n][K+2] = center, input, negs (-1 = negative equal to center) for
 * jobs [0, n_jobs); returns the number of records (may exceed cap). */
int64_t orc_sample_records(const int32_t *tok, const int64_t *sent_off, const int64_t *job_sent,
                           int64_t n_jobs, const uint64_t *job_seed, const uint32_t *sample_int,
                           int sample_on, const uint32_t *cum, int32_t V, int32_t K,
                           int32_t *rec_out, int64_t rec_cap) {
    int32_t *kept = (int32_t *)malloc(sizeof(int32_t) * MAX_SENTENCE_LEN);
    int32_t *sidx = (int32_t *)malloc(sizeof(int32_t) * (MAX_SENTENCE_LEN + 2));
    int64_t total = 0;
    for (int64_t j = 0; j < n_jobs; j++) {
        int64_t nex = 0;
        int32_t *dst = rec_out ? rec_out + total * (K + 2) : NULL;
        int64_t cap = rec_cap - total;
        train_job(tok, sent_off, job_sent[j], job_sent[j + 1], 0.0f, job_seed[j], sample_int,
                  sample_on, cum, V, NULL, NULL, NULL, 0, 0, K, NULL, kept, sidx, &nex,
                  cap > 0 ? dst : NULL, cap, 0, NULL, NULL);
        total += nex;
    }
    free(kept);
    free(sidx);
    return total;
}

/* explicit-negative steps: mode 0 = sequential (gensim order) */
void orc_sgns_step_sequential(float *syn0, float *syn1neg, const float *lockf, int64_t ld,
                              int32_t D, int32_t K, const int32_t *center, const int32_t *input,
                              const int32_t *negs, int64_t n, float alpha, float *loss) {
    ensure_exp();
    float *work = (float *)malloc(sizeof(float) * D);
    for (int64_t e = 0; e < n; e++)
        sg_neg(K, NULL, 0, syn0, syn1neg, ld, D, center[e], input[e], alpha, work, 0, lockf,
               negs + e * K, loss, NULL);
    free(work);
}
