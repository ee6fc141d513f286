/*
 * ORACLE (test infrastructure only): the pooling + cosine half of the CPU
 * checker, in plain C with OpenMP, for full-size (MIND-large dev, 376,471
 * impressions) parity checks where PyTorch's gather + index_add take minutes.
 *
 * Restates, over precomputed per-news tables (oracle/pool_ref.py
 * per_news_tables_large):
 *   FinalAttention pooling  modeling_utils.py:224-228
 *       u_d = sum_i x_{i,d} p_{i,d} / (sum_i p_{i,d} + 1e-10)   (rows hold [x*p | p])
 *   Latent pooling          latent_attention.py:165-170
 *       u = F.normalize(mean_i h_i, p=2, eps=1e-12)
 *   F.cosine_similarity     data_model_helper.py:223-227 (torch 2.10 per-vector clamp)
 *       s = (u / max(|u|, 1e-8)) . (e / max(|e|, 1e-8))
 * Sums run in double (the reference's f32 sums are order-dependent anyway; the
 * checker is pinned to oracle/pool_ref.cos_sim_scores_per_news, itself pinned to
 * the reference's golden vectors, in tests/test_oracle_golden.py).
 *
 * Built on first use by oracle/pool_ref.py (gcc -O3 -fopenmp -shared) into
 * oracle/libfastpool.so, and loaded by it only (test infrastructure).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#define DIM 1024

/* pooler 0 = FinalAttention (width 2048: [x*p | p]), 1 = Latent (width 1024).
 * users [n][1024] f32. */
void fp_pool(int pooler, const float* tab, int64_t width, const int64_t* hist_idx, const int64_t* hist_off, int64_t n,
             float* users) {
#pragma omp parallel
  {
    double* acc = (double*)malloc(sizeof(double) * 2 * DIM);
#pragma omp for schedule(dynamic, 64)
    for (int64_t i = 0; i < n; ++i) {
      const int64_t a = hist_off[i], b = hist_off[i + 1];
      const int k = pooler == 0 ? 2 : 1;
      for (int d = 0; d < k * DIM; ++d) acc[d] = 0.0;
      for (int64_t j = a; j < b; ++j) {
        const float* r = tab + hist_idx[j] * width;
        for (int d = 0; d < k * DIM; ++d) acc[d] += r[d];
      }
      float* u = users + i * DIM;
      if (pooler == 0) {
        for (int d = 0; d < DIM; ++d) u[d] = (float)(acc[d] / (acc[DIM + d] + 1e-10));
      } else {
        const double cnt = (double)(b - a);
        double ss = 0.0;
        for (int d = 0; d < DIM; ++d) {
          acc[d] /= cnt;
          ss += acc[d] * acc[d];
        }
        double nrm = sqrt(ss);
        if (nrm < 1e-12) nrm = 1e-12;
        for (int d = 0; d < DIM; ++d) u[d] = (float)(acc[d] / nrm);
      }
    }
    free(acc);
  }
}

/* scores[c] for candidates cand_off[i]..cand_off[i+1] of impression i against users[i]. */
void fp_cosine(const float* users, const float* table, const int64_t* cand_idx, const int64_t* cand_off, int64_t n,
               float* scores) {
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t i = 0; i < n; ++i) {
    const float* u = users + i * DIM;
    double uu = 0.0;
    for (int d = 0; d < DIM; ++d) uu += (double)u[d] * u[d];
    double un = sqrt(uu);
    if (un < 1e-8) un = 1e-8;
    for (int64_t c = cand_off[i]; c < cand_off[i + 1]; ++c) {
      const float* e = table + cand_idx[c] * DIM;
      double ee = 0.0, ue = 0.0;
      for (int d = 0; d < DIM; ++d) {
        ee += (double)e[d] * e[d];
        ue += (double)u[d] * e[d];
      }
      double en = sqrt(ee);
      if (en < 1e-8) en = 1e-8;
      scores[c] = (float)(ue / (un * en));
    }
  }
}
