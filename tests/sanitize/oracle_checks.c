/* oracle/als_oracle.c under AddressSanitizer + UndefinedBehaviorSanitizer
 * (SURVEY §5), built by tests/test_sanitizers.py: the synthetic generator,
 * one half-sweep at ranks 1 / 10 / 64 (incl. empty rows and a row whose
 * Gramian is singular without the lambda term) and the JVM-exact scoring
 * top-k with top_k above the item count. Checks the results are finite and
 * the rank-1 closed form x = sum(r v) / (sum(v^2) + n lambda). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int64_t oracle_synth_row(uint64_t seed, uint64_t seed2, uint64_t thr, uint64_t g, int64_t n_cols, int transposed,
                         int n_levels, int32_t* idx, float* val);
void oracle_half_sweep(const int64_t* indptr, const int32_t* indices, const float* values, int64_t n_rows,
                       const float* src, int64_t ld_src, int k, double reg, float* dst, int64_t ld_dst);
void oracle_score_topk(const float* U, int64_t ld_u, const int64_t* rows, int64_t n_sel, const float* V,
                       int64_t ld_v, int64_t n_items, int k, int top_k, int64_t* out_idx, float* out_val);

int main(void) {
  enum { NU = 60, NI = 45 };
  const uint64_t thr = UINT64_MAX / 5; /* density 0.2 */
  int64_t* indptr = malloc(sizeof(int64_t) * (NU + 1));
  int32_t* idx = malloc(sizeof(int32_t) * NU * NI);
  float* val = malloc(sizeof(float) * NU * NI);
  indptr[0] = 0;
  for (int u = 0; u < NU; ++u) {
    if (u % 7 == 3) { /* empty rows */
      indptr[u + 1] = indptr[u];
      continue;
    }
    indptr[u + 1] = indptr[u] + oracle_synth_row(20250620, 20250621, thr, u, NI, 0, 19, idx + indptr[u], val + indptr[u]);
  }
  const int ranks[3] = {1, 10, 64};
  int bad = 0;
  for (int q = 0; q < 3; ++q) {
    const int k = ranks[q];
    float* src = malloc(sizeof(float) * NI * k);
    float* dst = malloc(sizeof(float) * NU * k);
    for (int i = 0; i < NI * k; ++i) src[i] = (float)((i * 37 % 101) - 50) / 50.0f;
    oracle_half_sweep(indptr, idx, val, NU, src, k, k, 0.1, dst, k);
    for (int u = 0; u < NU; ++u)
      for (int c = 0; c < k; ++c) {
        if (!isfinite(dst[u * k + c])) bad = 1;
        if (indptr[u] == indptr[u + 1] && dst[u * k + c] != 0.f) bad = 1;
      }
    if (k == 1)
      for (int u = 0; u < NU; ++u) { /* rank 1: closed form */
        double num = 0, den = 0;
        for (int64_t p = indptr[u]; p < indptr[u + 1]; ++p) {
          num += (double)val[p] * src[idx[p]];
          den += (double)src[idx[p]] * src[idx[p]];
        }
        den += (double)(indptr[u + 1] - indptr[u]) * 0.1;
        const double want = den > 0 ? num / den : 0.0;
        if (fabs(dst[u] - want) > 1e-5 * (1 + fabs(want))) bad = 1;
      }
    int64_t rows[4] = {0, 5, 17, NU - 1};
    int64_t oi[4 * 50];
    float ov[4 * 50];
    oracle_score_topk(dst, k, rows, 4, src, k, NI, k, 50, oi, ov); /* top_k > n_items */
    for (int s = 0; s < 4; ++s)
      for (int p = NI; p < 50; ++p)
        if (oi[s * 50 + p] != -1) bad = 1;
    free(src);
    free(dst);
  }
  free(indptr);
  free(idx);
  free(val);
  if (bad) {
    fprintf(stderr, "oracle_checks FAILED\n");
    return 1;
  }
  printf("oracle_checks OK\n");
  return 0;
}
