/* g2v_train.c -- a host with no Python driving the C ABI (include/g2v.h):
 * one train() epoch of src/gene2vec.py:70's Word2Vec over a gene-pair corpus,
 * the way a C/C++ (or cgo / JNI) integration of libg2v.so would call it.
 *
 *   g2v_train <in.bin> <out.bin>
 *
 * in.bin (little-endian): int32 V, D, K, mode; int64 n_pairs, n_jobs;
 *   double alpha, min_alpha, sample; int64 counts[V] (vocabulary index order);
 *   float syn0[V*D] (initial vectors); int32 tokens[2*n_pairs];
 *   uint64 job_seed[n_jobs] (gensim's per-job model.random draws).
 * out.bin: float syn0[V*D], float syn1neg[V*D], g2v_stats.
 *
 * The per-job alphas follow [ext] _update_job_params for one epoch
 * (engine.job_alphas): alpha for the first job, then
 * max(min_alpha, alpha - (alpha - min_alpha) * pushed / n_pairs). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "g2v.h"

#define CHECK(call)                                                                   \
  do {                                                                                \
    int rc_ = (call);                                                                 \
    if (rc_ != G2V_OK) {                                                              \
      fprintf(stderr, "%s: %d (%s)\n", #call, rc_, g2v_last_error());                 \
      return 2;                                                                       \
    }                                                                                 \
  } while (0)

static int rd(FILE* f, void* p, size_t sz, size_t n) { return fread(p, sz, n, f) == n ? 0 : -1; }

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]);
    return 1;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 1;
  int32_t hdr[4];
  int64_t nn[2];
  double hp[3];
  if (rd(f, hdr, 4, 4) || rd(f, nn, 8, 2) || rd(f, hp, 8, 3)) return 1;
  const int32_t V = hdr[0], D = hdr[1], K = hdr[2];
  const uint32_t mode = (uint32_t)hdr[3];
  const int64_t n_pairs = nn[0], n_jobs_in = nn[1];
  int64_t* counts = malloc(sizeof(int64_t) * V);
  float* syn0 = malloc(sizeof(float) * (size_t)V * D);
  float* syn1 = calloc((size_t)V * D, sizeof(float));
  int32_t* tok = malloc(sizeof(int32_t) * 2 * (size_t)n_pairs);
  uint64_t* seed = malloc(sizeof(uint64_t) * (size_t)n_jobs_in);
  if (!counts || !syn0 || !syn1 || !tok || !seed) return 1;
  if (rd(f, counts, 8, V) || rd(f, syn0, 4, (size_t)V * D) || rd(f, tok, 4, 2 * (size_t)n_pairs) ||
      rd(f, seed, 8, (size_t)n_jobs_in))
    return 1;
  fclose(f);
  if (g2v_abi_version() != G2V_ABI_VERSION) {
    fprintf(stderr, "libg2v ABI %d, header %d\n", g2v_abi_version(), G2V_ABI_VERSION);
    return 2;
  }

  /* gensim's job producer over fixed-length (pair) sentences */
  int64_t n_jobs = 0;
  CHECK(g2v_plan_jobs(NULL, n_pairs, 2, G2V_BATCH_WORDS, NULL, 0, &n_jobs));
  if (n_jobs != n_jobs_in) {
    fprintf(stderr, "expected %lld job seeds, got %lld\n", (long long)n_jobs,
            (long long)n_jobs_in);
    return 2;
  }
  int64_t* job_sent = malloc(sizeof(int64_t) * (size_t)(n_jobs + 1));
  float* job_alpha = malloc(sizeof(float) * (size_t)(n_jobs > 0 ? n_jobs : 1));
  CHECK(g2v_plan_jobs(NULL, n_pairs, 2, G2V_BATCH_WORDS, job_sent, n_jobs + 1, &n_jobs));
  for (int64_t j = 0; j < n_jobs; ++j) {
    double a = hp[0];
    if (j > 0) {
      const double progress = (0.0 + 1.0 * (double)(job_sent[j] - job_sent[0]) / (double)n_pairs);
      a = hp[0] - (hp[0] - hp[1]) * progress;
      if (a < hp[1]) a = hp[1];
    }
    job_alpha[j] = (float)a;
  }

  g2v_ctx* ctx = NULL;
  CHECK(g2v_create(0, V, D, K, 1, &ctx));
  CHECK(g2v_set_vocab(ctx, counts, hp[2], 0.75, NULL, NULL));
  CHECK(g2v_set_weights(ctx, syn0, syn1, NULL));
  CHECK(g2v_set_corpus(ctx, tok, 2 * n_pairs, NULL, n_pairs, 2, 0));
  CHECK(g2v_train(ctx, job_sent, job_alpha, seed, n_jobs, mode));
  CHECK(g2v_get_weights(ctx, syn0, syn1));
  g2v_stats st;
  CHECK(g2v_read_stats(ctx, &st));
  CHECK(g2v_destroy(ctx));

  FILE* o = fopen(argv[2], "wb");
  if (!o) return 1;
  fwrite(syn0, sizeof(float), (size_t)V * D, o);
  fwrite(syn1, sizeof(float), (size_t)V * D, o);
  fwrite(&st, sizeof st, 1, o);
  fclose(o);
  printf("trained %lld pairs: %lld jobs, %lld effective words, %lld examples\n",
         (long long)n_pairs, (long long)st.jobs, (long long)st.effective_words,
         (long long)st.examples);
  free(counts); free(syn0); free(syn1); free(tok); free(seed); free(job_sent); free(job_alpha);
  return 0;
}
