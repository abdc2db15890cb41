/*
 * als_oracle.c — C restatement of Spark 3.5.1 explicit ALS per-row update,
 * TEST INFRASTRUCTURE ONLY (the CPU checker and the bench's cpu_baseline;
 * see oracle/__init__.py). Never linked into libhrec.
 *
 * Follows org.apache.spark.ml.recommendation.ALS [ext, pyspark 3.5.1,
 * requirements.txt:1; called from src/als_model.py:62]:
 *   NormalEquation.add   : dspr('U', k, 1.0, da, ata) ; if (r != 0) daxpy
 *   CholeskySolver.solve : ata[diag] += n * reg ; dppsv('U') ; toFloat
 * dppsv = dpptrf (left-looking packed Cholesky, netlib order) + dpptrs
 * (two packed triangular solves), restated from the netlib reference.
 * Also restates the synthetic matrix generator of BASELINE.md §3 so the CPU
 * baseline runs on the same matrix as the GPU.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

static uint64_t pair_hash(uint64_t seed, uint64_t u, uint64_t i) {
  return mix64(seed * 0x9E3779B97F4A7C15ull + ((u << 32) | (i & 0xffffffffull)));
}

/* One row (global id g) of R (transposed=0: user row over items) or R^T.
 * Writes column ids / ratings (may be NULL to count only); returns count. */
int64_t oracle_synth_row(uint64_t seed, uint64_t seed2, uint64_t thr, uint64_t g, int64_t n_cols,
                         int transposed, int n_levels, int32_t* idx, float* val) {
  int64_t cnt = 0;
  for (int64_t c = 0; c < n_cols; ++c) {
    const uint64_t u = transposed ? (uint64_t)c : g;
    const uint64_t i = transposed ? g : (uint64_t)c;
    if (pair_hash(seed, u, i) < thr) {
      if (idx) idx[cnt] = (int32_t)c;
      if (val) val[cnt] = (float)(pair_hash(seed2, u, i) % (uint64_t)n_levels);
      ++cnt;
    }
  }
  return cnt;
}

/* netlib dpptrf('U') on column-major packed upper ap (order k); 0 = ok. */
static int dpptrf_upper(int k, double* ap) {
  int jj = 0; /* 0-based index of diagonal (j,j) after update */
  for (int j = 0; j < k; ++j) {
    const int jc = jj; /* start of column j */
    jj += j + 1;       /* one past (j,j): diag at jj-1 */
    /* dtpsv('U','T','N', j, ap, ap+jc): solve U(0:j,0:j)^T x = ap[jc..] */
    for (int i = 0; i < j; ++i) {
      double t = ap[jc + i];
      const int ic = i * (i + 1) / 2; /* column i start */
      for (int q = 0; q < i; ++q) t -= ap[ic + q] * ap[jc + q];
      ap[jc + i] = t / ap[ic + i];
    }
    double d = 0.0;
    for (int q = 0; q < j; ++q) d += ap[jc + q] * ap[jc + q];
    const double ajj = ap[jj - 1] - d;
    if (!(ajj > 0.0)) return j + 1;
    ap[jj - 1] = sqrt(ajj);
  }
  return 0;
}

/* dpptrs('U', nrhs=1): U^T y = b, then U x = y (in place). */
static void dpptrs_upper(int k, const double* ap, double* b) {
  for (int i = 0; i < k; ++i) { /* U^T y = b: column i of U = ap[ic..ic+i] */
    const int ic = i * (i + 1) / 2;
    double t = b[i];
    for (int q = 0; q < i; ++q) t -= ap[ic + q] * b[q];
    b[i] = t / ap[ic + i];
  }
  for (int i = k - 1; i >= 0; --i) { /* U x = y, column oriented */
    const int ic = i * (i + 1) / 2;
    b[i] /= ap[ic + i];
    const double xi = b[i];
    for (int q = 0; q < i; ++q) b[q] -= ap[ic + q] * xi;
  }
}

/* One computeFactors pass over n_rows CSR rows. src/dst have leading dims
 * ld_src / ld_dst (>= k). Rows without ratings get zeros. */
void oracle_half_sweep(const int64_t* indptr, const int32_t* indices, const float* values,
                       int64_t n_rows, const float* src, int64_t ld_src, int k, double reg,
                       float* dst, int64_t ld_dst) {
  const int tri = k * (k + 1) / 2;
#pragma omp parallel
  {
    double* ata = (double*)malloc(sizeof(double) * (size_t)tri);
    double* atb = (double*)malloc(sizeof(double) * (size_t)k);
    double* da = (double*)malloc(sizeof(double) * (size_t)k);
#pragma omp for schedule(dynamic, 16)
    for (int64_t r = 0; r < n_rows; ++r) {
      float* out = dst + r * ld_dst;
      const int64_t b = indptr[r], e = indptr[r + 1];
      if (b == e) {
        for (int c = 0; c < k; ++c) out[c] = 0.f;
        continue;
      }
      memset(ata, 0, sizeof(double) * (size_t)tri);
      memset(atb, 0, sizeof(double) * (size_t)k);
      for (int64_t p = b; p < e; ++p) {
        const float* v = src + (int64_t)indices[p] * ld_src;
        for (int c = 0; c < k; ++c) da[c] = (double)v[c];
        /* dspr upper: column j gets x[0..j] * x[j] */
        int kk = 0;
        for (int j = 0; j < k; ++j) {
          const double t = da[j];
          if (t != 0.0)
            for (int i = 0; i <= j; ++i) ata[kk + i] += da[i] * t;
          kk += j + 1;
        }
        const double rating = (double)values[p];
        if (rating != 0.0)
          for (int c = 0; c < k; ++c) atb[c] += rating * da[c];
      }
      const double lambda = (double)(e - b) * reg;
      for (int i = 0, j = 2; i < tri; i += j, ++j) ata[i] += lambda;
      if (dpptrf_upper(k, ata) != 0) {
        for (int c = 0; c < k; ++c) out[c] = NAN;
        continue;
      }
      dpptrs_upper(k, ata, atb);
      for (int c = 0; c < k; ++c) out[c] = (float)atb[c];
    }
    free(ata);
    free(atb);
    free(da);
  }
}

int oracle_max_threads(void) {
#ifdef _OPENMP
  extern int omp_get_max_threads(void);
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* Spark ALSModel.transform's predict [ext: ALSModel.scala, called from
 * src/als_model.py:75]: `dot = 0f; for i < rank: dot += a(i) * b(i)` in f32,
 * product and sum each rounded (no FMA: built with -ffp-contract=off), then
 * Python's stable sorted(reverse=True)[:top_k] (src/hybrid_system.py:108):
 * ties keep the earlier item. One user row per OpenMP iteration; 8 items are
 * scored side by side (same per-item operation order, so still exact).
 * U: [n_sel rows gathered by `rows`, ld_u], V: [n_items, ld_v]. */
void oracle_score_topk(const float* U, int64_t ld_u, const int64_t* rows, int64_t n_sel, const float* V,
                       int64_t ld_v, int64_t n_items, int k, int top_k, int64_t* out_idx, float* out_val) {
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t s = 0; s < n_sel; ++s) {
    const float* u = U + rows[s] * ld_u;
    int64_t* oi = out_idx + s * top_k;
    float* ov = out_val + s * top_k;
    int filled = 0;
    for (int64_t j0 = 0; j0 < n_items; j0 += 8) {
      const int nb = (int)((n_items - j0) < 8 ? (n_items - j0) : 8);
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int c = 0; c < k; ++c) {
        const float a = u[c];
        for (int t = 0; t < nb; ++t) acc[t] = acc[t] + a * V[(j0 + t) * ld_v + c];
      }
      for (int t = 0; t < nb; ++t) {
        const float x = acc[t];
        if (filled == top_k && !(x > ov[top_k - 1])) continue;
        int p = filled < top_k ? filled++ : top_k - 1;
        while (p > 0 && x > ov[p - 1]) {
          ov[p] = ov[p - 1];
          oi[p] = oi[p - 1];
          --p;
        }
        ov[p] = x;
        oi[p] = j0 + t;
      }
    }
    for (int p = filled; p < top_k; ++p) {
      ov[p] = -INFINITY;
      oi[p] = -1;
    }
  }
}
