/*
 * hrec.h — C-ABI of libhrec.so, the MI355X (gfx950) hot path of the hybrid
 * ALS + two-tower recommender.
 *
 * The reference (HSoumi/hybrid-als-twotower-recommender) has no FFI of its
 * own: its hot path sits behind two third-party engines that its Python
 * wrappers call. Each entry point below replaces one of those downward calls
 * (file:line into the reference tree):
 *
 *   Spark  ALS.fit            src/als_model.py:52-62   -> hrec_synth_* (data),
 *                                                          hrec_als_init_factors,
 *                                                          hrec_als_half_sweep
 *   Spark  ALSModel.transform src/als_model.py:71-76   -> hrec_als_score
 *   Python/sklearn fusion     src/hybrid_system.py:57-75,108 -> hrec_fuse_topk
 *   Keras  two-tower graph    src/two_tower_model.py:38-89 -> hrec_tt_*
 *
 * Conventions (all functions):
 *   - every pointer is a DEVICE pointer owned by the caller, except where a
 *     parameter is documented as host memory;
 *   - row-major storage; factor matrices have a leading dimension `kp`
 *     (16, 32, 64, 96, 128, 192 or 256) >= k whose padding columns are kept
 *     at zero (kp > 64: one workgroup per row, csrc/als_wide.hip);
 *   - CSR: int64 indptr[n_rows+1] (local, starts at 0), int32 indices,
 *     f32 values;
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream);
 *     calls are asynchronous on it and never allocate or synchronise;
 *   - return 0 on success, a negative HREC_E* code on failure; the message
 *     of the last failure on the calling thread is hrec_last_error().
 */
#ifndef HREC_H
#define HREC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: hrec_fuse_topk gained out_minmax; hrec_hybrid_scores gained n_als_rows.
 * 3: hrec_hybrid_minmax / hrec_hybrid_topk removed (the pruned hybrid
 *    replaces them); hrec_dot_topk's +inf bound admits scores >= +inf.
 * 4: the RCCL exchange steps (hrec_comm_*, hrec_allgather, hrec_allreduce_minmax).
 * 6: hrec_als_score_topk_pruned_counts, hrec_cold_fallback*; the pruned ALS
 *    bound is 2^-7 + 2^-13 and its top_k <= 8 results are exact without a
 *    host-side fallback.
 * 7: hrec_encode_ids_ex (the ids' order from the marking pass). */
#define HREC_ABI_VERSION 7

#define HREC_OK 0
#define HREC_E_INVALID (-1) /* bad argument (shape, null pointer, range) */
#define HREC_E_LAUNCH (-2)  /* HIP launch/runtime error                  */
#define HREC_E_UNSUPPORTED (-3)

int hrec_abi_version(void);
const char* hrec_last_error(void);

/* ---------------------------------------------------------------- synth --
 * Synthetic interaction matrix R: (u,i) in R  <=>
 *   h64(seed,u,i) < threshold,  rating(u,i) = h64(seed2,u,i) mod n_levels,
 * h64(s,u,i) = mix64(s*0x9E3779B97F4A7C15 + (u<<32 | i)), mix64 = splitmix64
 * finaliser. The same predicate generates CSR rows (users, transposed=0) and
 * CSC columns (items, transposed=1) independently, so shards agree.
 * Rows are row_begin .. row_begin+n_rows-1 of the chosen orientation; the
 * other dimension has n_cols entries. Replaces the dataset the reference
 * reads at src/data_preprocessing.py:22-35 for the perf configurations. */
int hrec_synth_row_counts(uint64_t seed, uint64_t threshold, int64_t row_begin,
                          int64_t n_rows, int64_t n_cols, int transposed,
                          int64_t* counts, void* stream);
int hrec_synth_fill(uint64_t seed, uint64_t seed2, uint64_t threshold,
                    int64_t row_begin, int64_t n_rows, int64_t n_cols,
                    int transposed, int n_levels, const int64_t* indptr,
                    int32_t* indices, float* values, void* stream);

/* Exclusive prefix sum of counts[n] into out[n+1] (out[n] = total).
 * Workspace: hrec_scan_workspace_bytes(n) bytes of device memory. */
size_t hrec_scan_workspace_bytes(int64_t n);
int hrec_exclusive_scan_i64(const int64_t* counts, int64_t n, int64_t* out,
                            void* workspace, size_t workspace_bytes,
                            void* stream);

/* --------------------------------------------------------------- ingest --
 * The DataFrame -> CSR/CSC step of ALSModel.train (src/als_model.py:51-62:
 * Spark keys factors by the integer ids and keeps duplicate (user, item)
 * ratings as separate terms).
 *
 * hrec_minmax_i64: out[0] = min(x), out[1] = max(x) (device), n >= 1.
 * Workspace: hrec_minmax_i64_workspace_bytes(n). */
size_t hrec_minmax_i64_workspace_bytes(int64_t n);
int hrec_minmax_i64(const int64_t* x, int64_t n, int64_t* out, void* workspace,
                    size_t workspace_bytes, void* stream);

/* hrec_encode_ids: ids[n] (int64, id_lo <= ids <= id_hi) -> uniq[*n_uniq]
 * ascending distinct ids and codes[n] (int32 index into uniq), i.e.
 * numpy.unique(ids, return_inverse=True). *n_uniq is written on the device.
 * A range id_hi - id_lo < 2^31 sorts 32-bit keys on only the bits it spans;
 * pass INT64_MIN, INT64_MAX when the range is unknown. n < 2^31.
 * Workspace: hrec_encode_ids_workspace_bytes(n). */
size_t hrec_encode_ids_workspace_bytes(int64_t n);
int hrec_encode_ids(const int64_t* ids, int64_t n, int64_t id_lo, int64_t id_hi,
                    int64_t* uniq, int64_t* n_uniq, int32_t* codes,
                    void* workspace, size_t workspace_bytes, void* stream);
/* The same, plus *descending (device int32, may be null) = 1 if some
 * ids[i] > ids[i+1], else 0 — hrec_rows_descending_pairs of the codes
 * (the code map is monotone), read by the dense paths' marking pass instead
 * of a pass over the codes — and, when descending is 0, starts[0..n_uniq]
 * (may be null; room for min(n, id_hi - id_lo + 1) + 1 entries) = the CSR
 * row pointer of rows = codes, written by the code pass: ratings grouped by
 * user need neither hrec_rows_descending_pairs nor hrec_coo_to_csr_sorted
 * (the CSR is (starts, item codes, ratings)). starts needs descending. */
int hrec_encode_ids_ex(const int64_t* ids, int64_t n, int64_t id_lo, int64_t id_hi,
                       int64_t* uniq, int64_t* n_uniq, int32_t* codes,
                       int32_t* descending, int64_t* starts, void* workspace,
                       size_t workspace_bytes, void* stream);

/* hrec_coo_to_csr: (rows[nnz], cols[nnz], vals[nnz]) with 0 <= rows < n_rows
 * -> indptr[n_rows+1], indices[nnz], values[nnz]; rows ascending, the entries
 * of a row in input order (numpy.argsort(rows, kind="stable")). The CSC is
 * the same call with rows and cols swapped. nnz, n_rows < 2^31. The entries
 * ride the radix sort as 64-bit (col, rating) values (no gather after it).
 * Workspace: hrec_coo_to_csr_workspace_bytes(nnz, n_rows). */
size_t hrec_coo_to_csr_workspace_bytes(int64_t nnz, int64_t n_rows);
int hrec_coo_to_csr(const int32_t* rows, const int32_t* cols, const float* vals,
                    int64_t nnz, int64_t n_rows, int64_t* indptr, int32_t* indices,
                    float* values, void* workspace, size_t workspace_bytes,
                    void* stream);
/* The same CSR when rows[] is already non-decreasing (then input order is the
 * stable order): entries copied, indptr from the rows, no sort or workspace.
 * indices == cols and values == vals (both or neither) skip the copy: the
 * CSR's column and value arrays are then the input columns themselves.
 * hrec_rows_descending_pairs writes *out (device int32) = 1 if some
 * rows[i] > rows[i+1], else 0 — the caller's choice between the two. */
int hrec_rows_descending_pairs(const int32_t* rows, int64_t n, int32_t* out, void* stream);
int hrec_coo_to_csr_sorted(const int32_t* rows, const int32_t* cols, const float* vals,
                           int64_t nnz, int64_t n_rows, int64_t* indptr, int32_t* indices,
                           float* values, void* stream);

/* hrec_remap_i32: x[i] = table[x[i]] in place (ids outside [0, table_n)
 * -> -1). Maps an ALS shard's column ids (global user / item rows) to rows
 * of an nnz-balanced, padded factor layout (src/als_engine.py RowLayout;
 * Spark partitions users/items into numUserBlocks/numItemBlocks blocks
 * [ext: ALS.scala] — here contiguous row ranges balanced by ratings). */
int hrec_remap_i32(int32_t* x, int64_t n, const int32_t* table, int64_t table_n, void* stream);

/* ------------------------------------------------------------------ ALS --
 * Initial factors (Spark ALS.initialize [ext: pyspark 3.5.1 ALS.scala]:
 * per row a Gaussian-like vector, L2-normalised, f32). Counter-based on
 * (seed, global row) so every shard layout yields the same matrix. */
int hrec_als_init_factors(uint64_t seed, int64_t row_begin, int64_t n_rows,
                          int k, int kp, float* out, void* stream);

/* One ALS half-sweep (Spark computeFactors + NormalEquation.add +
 * CholeskySolver.solve [ext]; called from src/als_model.py:62):
 * for every local dst row r with n_r = indptr[r+1]-indptr[r] ratings,
 *   (sum_j v_j v_j^T + reg_param*n_r*I) x_r = sum_j rating_j v_j,
 * v_j = src_factors[indices[j]], accumulated in f64 (accum_mode 0), solved
 * by Cholesky in f64, stored as f32 in dst_factors[r*kp .. +kp).
 * Rows with n_r == 0 get a zero vector (Spark has no factor for them).
 * accum_mode: 0 = Gramian accumulated in f64 on the f64 matrix cores
 *             (Spark's f64 NormalEquation);
 *             1 = f32 matrix-core products summed in f32 within chunks of 16
 *             ratings, chunks summed in f64 (2x the matrix rate; parity
 *             checked at rtol 1e-4 in tests/test_gpu_core.py). */
int hrec_als_half_sweep(const int64_t* indptr, const int32_t* indices,
                        const float* values, int64_t n_rows,
                        const float* src_factors, int64_t n_src, int k, int kp,
                        double reg_param, int accum_mode, float* dst_factors,
                        void* stream);

/* The same half-sweep with the source factors given in f64
 * (src64[n_src*kp] = the f32 factors converted exactly, hrec_f32_to_f64):
 * identical results, no per-step f32 -> f64 conversion in the gather. For
 * sources that stay in the MI355X's on-chip caches (the user side at
 * BASELINE c2: 100k item rows = 51 MB in f64). kp = 64, accum_mode 0. */
int hrec_als_half_sweep_src64(const int64_t* indptr, const int32_t* indices, const float* values,
                              int64_t n_rows, const double* src64, int64_t n_src, int k, int kp,
                              double reg_param, float* dst_factors, void* stream);
/* out[i] = (double)in[i]. */
int hrec_f32_to_f64(const float* in, int64_t n, double* out, void* stream);

/* out[c*ld_out + r] = in[r*cols + c] (f32), ld_out >= rows. */
int hrec_transpose_f32(const float* in, int64_t rows, int64_t cols, float* out,
                       int64_t ld_out, void* stream);

/* ALS scoring (Spark ALSModel.transform predict UDF [ext], reached from
 * src/als_model.py:75): out[b*n_items + j] = sum_{c<k} U[u_b][c]*V[i_j][c]
 * as a sequential f32 chain, product rounded then sum rounded (no FMA),
 * exactly the JVM loop. NaN where u_b < 0 or i_j < 0 (unknown id).
 * user_factors is [*, kp] row-major; item_factors_t is the TRANSPOSED item
 * matrix [kp, ld_items]; item_rows == NULL means i_j = j. */
int hrec_als_score(const float* user_factors, const int64_t* user_rows,
                   int n_users, const float* item_factors_t, int64_t ld_items,
                   const int64_t* item_rows, int64_t n_items, int k, int kp,
                   float* out, void* stream);

/* Scoring consumed by a top-k, for whole item ranges (no id gather): the
 * same JVM-exact f32 dot as hrec_als_score for every (user, item j < n_items)
 * pair, but the B x n_items score matrix is never written: the top_k-th
 * best score of the first 2048 items bounds each user's final top_k-th score
 * from below, a fused pass keeps only pairs at or above that bound, and an
 * exact stable top-k runs over the survivors. out_idx/out_val: [n_users,
 * min(top_k, n_items)]. *overflow (device int) is set to 1 when some user had
 * more than 4096 survivors (ties/adversarial scores): the result is then
 * incomplete and the caller must fall back to hrec_als_score + hrec_topk_f32.
 * Users must be known (user_rows >= 0). ld_items % 4 == 0. */
size_t hrec_als_score_topk_workspace_bytes(int n_users, int64_t n_items, int top_k);
int hrec_als_score_topk(const float* user_factors, const int64_t* user_rows,
                        int n_users, const float* item_factors_t, int64_t ld_items,
                        int64_t n_items, int k, int kp, int top_k, int64_t* out_idx,
                        float* out_val, int* overflow, void* workspace,
                        size_t workspace_bytes, void* stream);

/* Pruned form of hrec_als_score_topk (same outputs, same overflow contract):
 * the sample bound thr_b as there, then a bf16 matrix-core filter keeps
 * every item with approx score >= thr_b - E, E = (2^-7 + 2^-13) ||u|| max
 * ||v|| + 1e-30 (bounds |bf16 dot - JVM chain| for k <= 256: 2^-8 relative
 * rounding per bf16 operand), and the JVM chain over those items alone
 * leaves exactly the fused filter's survivors (score >= thr_b), ranked by the
 * same stable top-k. *overflow is also set when a bound is not finite (a
 * non-finite factor), when the bf16 filter's list overflows, or when a known
 * user ends with fewer than min(top_k, n_items) candidates (a bound slip:
 * never short or padded ids). For min(top_k, n_items) <= 8 a set *overflow
 * is resolved in the same call, on the device (a gated exact top-k of the
 * JVM chain over every item, no host round trip): the outputs are then
 * always exact and *overflow only reports that the fallback ran; above 8 the
 * caller falls back as for hrec_als_score_topk. items_bf16: hrec_als_items_bf16 of
 * item_factors (row-major [n_items, ld_v], the same values as
 * item_factors_t), 256-B aligned; it is built once per item matrix.
 * hrec_als_score_topk_pruned_counts copies the last call's diagnostics from
 * its workspace: out[0 .. n) = pairs the bf16 bound kept per user,
 * out[n .. 2n) = candidates per user (int32, device); zeros when the call
 * took the small-catalogue (fused) path. */
size_t hrec_als_items_bf16_bytes(int64_t n_items, int k);
int hrec_als_items_bf16(const float* item_factors, int64_t ld_v, int64_t n_items, int k,
                        void* out, size_t out_bytes, void* stream);
size_t hrec_als_score_topk_pruned_workspace_bytes(int n_users, int64_t n_items, int top_k, int k);
int hrec_als_score_topk_pruned(const float* user_factors, const int64_t* user_rows, int n_users,
                               const float* item_factors_t, int64_t ld_items,
                               const float* item_factors, int64_t ld_v, const void* items_bf16,
                               int64_t n_items, int k, int kp, int top_k, int64_t* out_idx,
                               float* out_val, int* overflow, void* workspace,
                               size_t workspace_bytes, void* stream);
int hrec_als_score_topk_pruned_counts(const void* workspace, int n_users, int64_t n_items, int top_k, int k,
                                      int32_t* out, void* stream);

/* ---------------------------------------------------------------- top-k --
 * Stable descending top-k of each of n_rows rows (row i starts at
 * vals + i*row_stride, n elements): larger value first, equal values keep
 * input order (smaller index first), NaN last — Python's
 * sorted(..., key=score, reverse=True)[:k] as used at
 * src/hybrid_system.py:108 and src/als_model.py:173. Any top_k >= 1 (clamped
 * to n): up to 1024 by segment selections, above by a stable per-row radix
 * sort on the device (then n_rows * n < 2^31). */
size_t hrec_topk_workspace_bytes(int64_t n_rows, int64_t n, int top_k, int is_f64);
int hrec_topk_f32(const float* vals, int64_t n_rows, int64_t n, int64_t row_stride,
                  int top_k, int64_t* out_idx, float* out_val, void* workspace,
                  size_t workspace_bytes, void* stream);
int hrec_topk_f64(const double* vals, int64_t n_rows, int64_t n, int64_t row_stride,
                  int top_k, int64_t* out_idx, double* out_val, void* workspace,
                  size_t workspace_bytes, void* stream);

/* --------------------------------------------------------------- fusion --
 * HybridRecommendationSystem.adaptive_fusion + top-k
 * (src/hybrid_system.py:57-75 and :108): both score vectors (aligned to the
 * same item order) are min-max scaled with sklearn MinMaxScaler arithmetic
 * in their own dtype (als f64; tt f32 when tt_is_f32, else f64), then
 * fused = w0*als_norm + w1*tt_norm in f64 with (w0,w1) = (0.8,0.2) when
 * als_wins (the strict als_f1 > tt_f1 of :69) else (0.2,0.8).
 * out_fused (optional, n doubles) receives every fused score; out_idx /
 * out_score receive the stable top min(top_k, n) (any top_k >= 0; 0 = no
 * top-k). out_minmax (optional, 4 doubles) receives (als min, als max,
 * tt min, tt max): the two scalers' data_min_ / data_max_ after the
 * reference's fit_transform (src/hybrid_system.py:66-67). */
size_t hrec_fuse_workspace_bytes(int64_t n, int top_k);
int hrec_fuse_topk(const double* als, const void* tt, int tt_is_f32, int64_t n,
                   int als_wins, int top_k, int64_t* out_idx, double* out_score,
                   double* out_fused, double* out_minmax, void* workspace,
                   size_t workspace_bytes, void* stream);

/* Batched fusion for many users over one item range (a shard of the item
 * set when the item rows are split across GPUs):
 * hrec_rows_minmax_f32: out[r] = min, out[n_rows + r] = max of row r (NaN
 * ignored) — reduced across shards by the caller (RCCL all-reduce MIN on the
 * first half, MAX on the second);
 * hrec_fuse_rows_topk: per row, MinMaxScaler of the ALS scores in f64 and of
 * the two-tower scores in f32 with the GIVEN (global) row min/max, f64 fusion
 * as hrec_fuse_topk, then the stable top-k of the row; indices are shifted by
 * idx_offset (the shard's first global item). als/tt: [n_rows, ld] f32.
 * hrec_topk_f64_keyed: stable top-k where keys[] (e.g. global item ids, -1 =
 * empty slot) are both the tie-break and the returned ids — the merge of the
 * per-shard candidates. */
int hrec_rows_minmax_f32(const float* x, int64_t n_rows, int64_t n, int64_t ld,
                         float* out, void* stream);
size_t hrec_fuse_rows_workspace_bytes(int64_t n_rows, int64_t n, int top_k);
int hrec_fuse_rows_topk(const float* als, const float* tt, int64_t n_rows, int64_t n,
                        int64_t ld, const float* als_minmax, const float* tt_minmax,
                        int als_wins, int top_k, int64_t idx_offset, int64_t* out_idx,
                        double* out_val, void* workspace, size_t workspace_bytes,
                        void* stream);
int hrec_topk_f64_keyed(const double* vals, const int64_t* keys, int64_t n_rows, int64_t n,
                        int top_k, int64_t* out_idx, double* out_val, void* workspace,
                        size_t workspace_bytes, void* stream);

/* ------------------------------------------------------ cold-start sim --
 * ALSModel._find_similar_items (src/als_model.py:93-104): out[q*n_items+j] =
 * cosine(feats[query_rows[q]], feats[j]) with sklearn's normalise-then-dot
 * (zero norm -> 1); the query's own entry is -inf (the reference skips it).
 * feats: [n_items, dim] f64 row-major in item_features dict order. */
int hrec_cosine_sim(const double* feats, int64_t n_items, int dim,
                    const int64_t* query_rows, int64_t n_query, double* out,
                    void* stream);

/* The cold-start fallback of EVERY item, once per model (src/als_model.py
 * :78-86 + _find_similar_items :93-104; the value depends on the item only):
 * out_mean[i] = the mean 'rating' (ratings[j], f64) of the <= 3 items j != i
 * most similar to i (hrec_cosine_sim's values, ranked larger first, ties ->
 * smaller j) with similarity > 0.5, as np.mean sums them ((r0 + r1) + r2) /
 * count; out_count[i] = how many (0: the caller's global mean; out_mean 0);
 * out_idx (optional, [n_items][3] int32, -1 padded) = those j in rank order.
 * feats [n_items][dim] f64 row-major, dim <= 16, n_items < 2^31. One pass of
 * n_items^2 similarities, no similarity matrix in memory.
 * Workspace: hrec_cold_fallback_workspace_bytes(n_items, dim). */
size_t hrec_cold_fallback_workspace_bytes(int64_t n_items, int dim);
int hrec_cold_fallback(const double* feats, const double* ratings, int64_t n_items, int dim,
                       double* out_mean, int32_t* out_count, int32_t* out_idx, void* workspace,
                       size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------ two-tower --
 * Keras graph of src/two_tower_model.py:38-89 (embedding_size d):
 *   user_vec = LN_u(E_user[u]);  h = relu(numeric @ W1 + b1)  [Dense(16)]
 *   z = [E_item[i] | E_man[m] (8) | E_cat[c] (8) | h (16)]    (d+32)
 *   item_vec = LN_i(z @ W2 + b2) [Dense(d)];  score = <user_vec, item_vec>
 * LayerNormalization: epsilon 1e-3, biased variance, y = xhat*gamma + beta.
 * All tensors f32 row-major on the device; ids int32 (< 2^24, see D11). */
typedef struct hrec_tt_params {
  int32_t d;
  int32_t reserved;
  float* user_emb;      /* [n_users, d]    */
  float* item_emb;      /* [n_items, d]    */
  float* man_emb;       /* [n_man, 8]      */
  float* cat_emb;       /* [n_cat, 8]      */
  float* w1;            /* [2, 16]         */
  float* b1;            /* [16]            */
  float* w2;            /* [d + 32, d]     */
  float* b2;            /* [d]             */
  float* ln_user_gamma; /* [d] */
  float* ln_user_beta;  /* [d] */
  float* ln_item_gamma; /* [d] */
  float* ln_item_beta;  /* [d] */
} hrec_tt_params;

/* Item tower over n candidate rows (the per-candidate graph evaluated by
 * model.predict at src/two_tower_model.py:145). */
int hrec_tt_item_forward(const hrec_tt_params* params, const int32_t* item,
                         const int32_t* manufacturer, const int32_t* category,
                         const float* numeric /* [n,2] */, int64_t n,
                         float* item_vec /* [n,d] */, void* stream);
/* User tower for n users. */
int hrec_tt_user_forward(const hrec_tt_params* params, const int32_t* user, int64_t n,
                         float* user_vec /* [n,d] */, void* stream);
/* Dot(axes=1) of every user row with every item row: out[b*n_items + j]
 * (f32). Every two-tower score in libhrec (this call at any n_users,
 * hrec_tt_pair_score, hrec_dot_scores / hrec_dot_topk on f32 operands, the
 * exact hybrid) is one fmaf chain from zero in one k order, so a score's bits
 * do not depend on the batch: d in {32, 64, 128, 256}: steps of 16, inside a
 * step k = 16 s + 4 g + e with g fastest (the v_mfma_f32_16x16x4_f32 tiles);
 * any other d: k = 0 .. d-1. */
int hrec_tt_score(const float* user_vec, int n_users, const float* item_vec,
                  int64_t n_items, int d, float* out, void* stream);

/* The item tower's inputs of one predict_for_user call from the candidate
 * frame's raw columns (src/two_tower_model.py:136-146): item / manufacturer /
 * category ids (int64) -> int32 (each in [0, its table) and below 2^24, where
 * Keras' float32 Input round trip is the identity), numeric [n,2] f32 =
 * (price, rating) * scale + min in f64 (MinMaxScaler.transform), rounded once.
 * scale / min_: HOST arrays of 2 doubles (the fitted scaler's scale_ / min_).
 * *flags (device int32, written by the call): bit 1 an id outside those
 * bounds, bit 2 an infinite numeric input, bit 4 a repeated item id — the
 * outputs are then unusable and the caller takes the host path (which raises
 * the reference's error where it raises). Replaces the host-side _ids casts,
 * scaler.transform and the candidate-uniqueness pass of the hybrid's array
 * path (src/hybrid_system.py:95-116). */
size_t hrec_tt_item_inputs_workspace_bytes(int64_t n_item_table);
int hrec_tt_item_inputs(const int64_t* item, const int64_t* manufacturer, const int64_t* category,
                        const double* price, const double* rating, int64_t n, int64_t n_item_table,
                        int64_t n_man_table, int64_t n_cat_table, const double* scale, const double* min_,
                        int32_t* item_out, int32_t* man_out, int32_t* cat_out, float* numeric_out,
                        int32_t* flags, void* workspace, size_t workspace_bytes, void* stream);

/* Row-wise dot: out[r] = <user_vec[r], item_vec[r]> (n rows of d), in
 * hrec_tt_score's order (the same bits for the same pair). */
int hrec_tt_pair_score(const float* user_vec, const float* item_vec, int64_t n, int d,
                       float* out, void* stream);

/* One minibatch of model.fit (src/two_tower_model.py:111): forward, MSE
 * loss, backward. grad_dense receives hrec_tt_grad_len(d) floats:
 * dW2[(d+32)*d] | db2[d] | dgamma_i[d] | dbeta_i[d] | dgamma_u[d] | dbeta_u[d]
 * | dW1[32] | db1[16] | sum_sq_err[1] | sum_abs_err[1]  (loss = sum_sq_err/batch).
 * g_user/g_item [batch,d], g_man/g_cat [batch,8]: per-sample embedding-row
 * gradients (IndexedSlices values, duplicates not yet summed). */
size_t hrec_tt_train_workspace_bytes(int d, int64_t batch);
size_t hrec_tt_grad_len(int d);
int hrec_tt_forward_backward(const hrec_tt_params* params, const int32_t* user,
                             const int32_t* item, const int32_t* manufacturer,
                             const int32_t* category, const float* numeric,
                             const float* y, int64_t batch, float* grad_dense,
                             float* g_user, float* g_item, float* g_man, float* g_cat,
                             void* workspace, size_t workspace_bytes, void* stream);

/* TF 2.8 ResourceApplyAdam (dense variables): m += (g-m)(1-b1);
 * v += (g^2-v)(1-b2); var -= m*alpha/(sqrt(v)+eps). alpha (host, f32) =
 * lr*sqrt(1-b2^t)/(1-b1^t). */
int hrec_adam_dense(float* var, float* m, float* v, const float* grad, int64_t n,
                    float alpha, float beta1, float beta2, float epsilon, void* stream);
/* Keras OptimizerV2 Adam._resource_apply_sparse on an embedding table:
 * duplicate indices summed in sample order (tf.unique + segment sum), then
 * m = m*b1 (whole table), m[idx] += g*(1-b1); v likewise with g^2; var -=
 * lr*m/(sqrt(v)+eps) over the WHOLE table. mark: int32[n_rows] all -1 on
 * entry (restored on exit); gsum: [batch, dim] scratch. */
int hrec_adam_sparse(float* var, float* m, float* v, int64_t n_rows, int dim,
                     const int32_t* indices, const float* grad_rows, int batch,
                     int32_t* mark, float* gsum, float lr, float beta1,
                     float one_minus_beta1, float beta2, float one_minus_beta2,
                     float epsilon, void* stream);

/* hrec_adam_sparse over several tables in one set of launches (the four
 * embedding tables of one Keras train step, src/two_tower_model.py:85,111):
 * per table exactly hrec_adam_sparse's arithmetic; 3 launches in total
 * instead of 3 per table. At most HREC_MAX_SPARSE_TABLES tables. */
#define HREC_MAX_SPARSE_TABLES 8
typedef struct hrec_sparse_table {
  float* var;
  float* m;
  float* v;
  int64_t n_rows;
  int32_t dim;
  int32_t batch;
  const int32_t* indices;
  const float* grad_rows;
  int32_t* mark;
  float* gsum;
} hrec_sparse_table;

int hrec_adam_sparse_tables(const hrec_sparse_table* tables, int n_tables, float lr,
                            float beta1, float one_minus_beta1, float beta2,
                            float one_minus_beta2, float epsilon, void* stream);

/* hrec_adam_sparse_tables in phases, for a two-stream train step: the
 * whole-table sweep of the rows the batch does NOT touch (phase 1, nearly all
 * of the step's HBM bytes) runs on a second stream beside the batch's
 * forward / backward, which read only touched rows; phase 2 then sums the
 * batch's gradients and steps the touched rows. Phases 0..3 in order give
 * bit for bit the rows of hrec_adam_sparse_tables (same Keras IndexedSlices
 * Adam, src/two_tower_model.py:111 via model.fit). Phase 1 may overlap phase
 * 2, never phase 0 or 3. Needs dim % 4 == 0 and 16-B aligned var/m/v; gsum
 * is not used, grad_rows only by phase 2. */
#define HREC_SPARSE_MARK 0
#define HREC_SPARSE_SWEEP_UNTOUCHED 1
#define HREC_SPARSE_TOUCHED 2
#define HREC_SPARSE_UNMARK 3
int hrec_adam_sparse_tables_phase(const hrec_sparse_table* tables, int n_tables, int phase,
                                  float lr, float beta1, float one_minus_beta1, float beta2,
                                  float one_minus_beta2, float epsilon, void* stream);

/* ---------------------------------------------------------------------
 * Matrix-core dot-product scoring + fused top-k (csrc/dot_topk.hip).
 * Replaces Keras Dot(axes=1) over every candidate in model.predict
 * (src/two_tower_model.py:80, :136-146) and the ranking after it
 * (sorted(..., reverse=True)[:k], src/hybrid_system.py:108), at BASELINE
 * configs c4 (d = 128, 50M candidates) and c5 (bf16, d = 256).
 * Operands: row-major [n, dk] with dk in {32, 64, 128, 256} (the model's d
 * zero-padded), 16-B aligned; dtype 0 = f32 (exact f32 fma chains on
 * v_mfma_f32_16x16x4_f32, k order permuted), 1 = bf16 bit patterns
 * (v_mfma_f32_16x16x32_bf16, f32 accumulation). n_items < 2^31. */
int hrec_f32_to_bf16(const float* in, int64_t n, uint16_t* out, void* stream);
/* out[b*ld_out + j] = <U[b], V[j]> for b < n_users, j < n_items.
 * Summation order and batch size: f32 calls of 1-4 users run the streaming
 * GEMV kernel, larger batches the matrix-core tiles; both issue the same
 * v_mfma_f32_16x16x4_f32 sequence per score (k order 16 ks + 4 g + e), so a
 * user's scores have the same bits at every batch size. bf16 calls always use
 * the matrix-core tiles. The same holds for hrec_dot_topk. */
int hrec_dot_scores(const void* user_vec, int n_users, const void* item_vec, int64_t n_items, int dk,
                    int dtype, float* out, int64_t ld_out, void* stream);
size_t hrec_dot_topk_workspace_bytes(int n_users, int64_t n_items, int top_k);
/* Stable top-k (larger first, ties -> smaller item index) of every user's
 * scores over items [0, n_items), without writing the score matrix: the
 * k-th best of a strided item sample (or thr_in[b] when thr_in != NULL) is a
 * lower bound of the k-th best; a fused score + filter pass appends the
 * survivors to a per-user list, ranked by an exact stable top-k. out_idx
 * gets idx_offset added (item shards). *overflow != 0 when a user had more
 * survivors than the list holds — then rerun with thr_in = out_val[:, k-1]
 * (the k-th best survivor is a higher valid bound). n_users < 65536. */
int hrec_dot_topk(const void* user_vec, int n_users, const void* item_vec, int64_t n_items, int dk,
                  int dtype, int top_k, const float* thr_in, int64_t idx_offset, int64_t* out_idx,
                  float* out_val, int* overflow, void* workspace, size_t workspace_bytes,
                  void* stream);
/* The survivor filter of hrec_dot_topk / the pruned hybrid alone: append
 * (score, j) of every item j with <U[b], V[j]> >= thr[b * thr_stride + (thr_per
 * ? j / thr_per : 0)] to user b's list (cand_val / cand_idx [n_users, cap]; a
 * NaN bound admits every score, a +inf bound none — a dead user or group,
 * skipped; hrec_dot_topk's own filter instead admits scores >= +inf for a
 * +inf bound; list order unspecified). cand_n[b], zeroed by
 * the caller, ends as the user's survivor count, or > cap when the list
 * overflowed (the list then holds an arbitrary subset). bf16 operands, or f32
 * at dk <= 128. */
int hrec_dot_filter(const void* user_vec, int n_users, const void* item_vec, int64_t n_items, int dk,
                    int dtype, const float* thr, int thr_stride, int64_t thr_per, int cap, float* cand_val,
                    int64_t* cand_idx, int* cand_n, void* stream);

/* ---------------------------------------------------------------------
 * Both score matrices of the bf16 hybrid in one launch (csrc/hybrid_scores.hip,
 * BASELINE config c5): the scores get_hybrid_recommendations ranks per user
 * (ALS transform + Keras Dot over every candidate, src/hybrid_system.py:95-116)
 * and the per-model MinMaxScaler extremes it fits (src/hybrid_system.py:57-75).
 * User rows are f32 (ALS: als_users[als_rows[b] * als_ld + c], als_rows may
 * be NULL for row b; a row outside [0, n_als_rows) — an unknown user — gives
 * a NaN score row, as hrec_als_score does for row -1, whose min / max are
 * +inf / -inf; two-tower: tt_users[b * tt_ld + c]), converted to bf16
 * (round to nearest even) for columns c < width and zero up to dk; item
 * operands are bf16 [n_items, dk], dk in {64, 128, 256}. Writes
 * als_out / tt_out [n_users, ld_out] f32 (bit-identical to hrec_dot_scores on
 * hrec_f32_to_bf16 operands) and als_mm / tt_mm [2, n_users] f32 =
 * hrec_rows_minmax_f32 of those rows. */
size_t hrec_hybrid_scores_workspace_bytes(int n_users, int64_t n_items);
int hrec_hybrid_scores(const float* als_users, int64_t als_ld, const int64_t* als_rows,
                       int64_t n_als_rows, int als_width,
                       const float* tt_users, int64_t tt_ld, int tt_width, int n_users,
                       const void* als_items, const void* tt_items, int64_t n_items, int dk,
                       float* als_out, float* tt_out, int64_t ld_out, float* als_mm, float* tt_mm,
                       void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------
 * Pruned bf16 hybrid top-k (csrc/hybrid_prune.hip, BASELINE config c5):
 * get_hybrid_recommendations for a batch of users over an item shard
 * (src/hybrid_system.py:57-75, :108) without writing either score matrix.
 * Same arguments as hrec_hybrid_scores for the users / items; results bit for
 * bit those of hrec_hybrid_scores + hrec_fuse_rows_topk.
 * Phase 1 (hrec_hybrid_prune_minmax): per-user [min | max] of both score rows
 *   into als_mm / tt_mm ([2, n_users] f32, the hrec_rows_minmax_f32 layout)
 *   and, in the workspace, each item group's maximum slice. With the items
 *   sharded, all-reduce the mins (MIN) and maxes (MAX) across shards before
 *   phase 2.
 * Phase 2 (hrec_hybrid_prune_topk): with the (global) min / max: a lower
 *   bound of each user's k-th best fused score from the group maxima, the
 *   heavier-weighted model's scores filtered against it, the survivors' other
 *   score and fused score, the stable top-k (ties -> smaller item; ids +
 *   idx_offset). Lists that overflow, users with non-finite scores or fewer
 *   survivors than k take the exact unfused path, gated on the device (no host
 *   round trip; hrec_hybrid_prune_fallback_taken copies that flag).
 * top_k in [1, 8]; the workspace (hrec_hybrid_prune_workspace_bytes, the same
 * dk and top_k) carries phase 1's state into phase 2: per item group G =
 * ceil(n_items / group) the group partials and arg-slices (24 B per user and
 * group), both bf16 user operands (4 dk B per user), the per-group bounds
 * (4 B per user and group) and each user's survivor list of 8192 entries
 * (96 KiB per user, whatever n_items is; the exact fallback runs inside the
 * survivor kernel and needs no score matrices). About 100 KiB per user at
 * c5: 25 MB for 256 users. n_users < 65536. */
size_t hrec_hybrid_prune_workspace_bytes(int n_users, int64_t n_items, int dk, int top_k);
int hrec_hybrid_prune_minmax(const float* als_users, int64_t als_ld, const int64_t* als_rows,
                             int64_t n_als_rows, int als_width, const float* tt_users, int64_t tt_ld,
                             int tt_width, int n_users, const void* als_items, const void* tt_items,
                             int64_t n_items, int dk, float* als_mm, float* tt_mm, void* workspace,
                             size_t workspace_bytes, void* stream);
int hrec_hybrid_prune_topk(const float* als_users, int64_t als_ld, const int64_t* als_rows,
                           int64_t n_als_rows, int als_width, const float* tt_users, int64_t tt_ld,
                           int tt_width, int n_users, const void* als_items, const void* tt_items,
                           int64_t n_items, int dk, const float* als_mm, const float* tt_mm, int als_wins,
                           int top_k, int64_t idx_offset, int64_t* out_idx, double* out_val,
                           void* workspace, size_t workspace_bytes, void* stream);
int hrec_hybrid_prune_fallback_taken(const void* workspace, int n_users, int64_t n_items, int dk,
                                     int top_k, int* out, void* stream);
/* Both phases for ONE item shard (no cross-shard min / max to combine): the
 * same results as hrec_hybrid_prune_minmax + hrec_hybrid_prune_topk (als_mm /
 * tt_mm are outputs here, [2, n_users] f32) with one launch fewer (the bound
 * kernel reduces the extremes). Same workspace. */
int hrec_hybrid_prune_local(const float* als_users, int64_t als_ld, const int64_t* als_rows, int64_t n_als_rows,
                            int als_width, const float* tt_users, int64_t tt_ld, int tt_width, int n_users,
                            const void* als_items, const void* tt_items, int64_t n_items, int dk, int als_wins,
                            int top_k, int64_t idx_offset, float* als_mm, float* tt_mm, int64_t* out_idx,
                            double* out_val, void* workspace, size_t workspace_bytes, void* stream);
/* Diagnostics of the last phase 2: the survivors of the heavy-model filter per
 * user (out: n_users int32, device). */
int hrec_hybrid_prune_survivors(const void* workspace, int n_users, int64_t n_items, int dk, int top_k,
                                int32_t* out, void* stream);

/* ---------------------------------------------------------------------
 * Exact hybrid top-k without score matrices (csrc/hybrid_exact.hip, BASELINE
 * config c2): get_hybrid_recommendations for a batch of users over an item
 * shard (src/hybrid_system.py:57-75, :95-116) with the reference's numerics —
 * the JVM-exact ALS dot (Spark ALSModel.transform, src/als_model.py:75) and
 * the f32 Keras Dot (src/two_tower_model.py:80) in hrec_dot_scores' MFMA k
 * order — bit for bit the result of hrec_als_score + hrec_tt_score (any
 * n_users >= 1) + hrec_rows_minmax_f32 + hrec_fuse_rows_topk, without writing either
 * [n_users, n_items] score matrix: both models are approximated on the bf16
 * matrix cores with a rigorous error bound, and only the item groups the
 * bound cannot rule out (a model's extremes; the fused top-k) are rescored
 * with the exact chains.
 *   als_users[als_rows[b] * als_ld + c], c < als_width (a row outside
 *     [0, n_als_rows) is an unknown user: NaN ALS scores);
 *   tt_users[b * tt_ld + c], c < tt_width in {32, 64, 128};
 *   als_items_t: the shard's ALS item factors transposed (item j, column c
 *     at als_items_t[c * als_items_ld + j]: hrec_als_score's layout);
 *   tt_items: the shard's two-tower item vectors, row-major (row stride a
 *     multiple of 4, 16-B aligned), tt_items_t the same transposed;
 *   prepared: hrec_hybrid_exact_prepare's split-bf16 operands + norm bounds
 *     of the same items (hrec_hybrid_exact_items_bytes, once per shard);
 *   dk in {64, 128} >= both widths. n_users < 65536. */
typedef struct hrec_hybrid_batch {
  const float* als_users;
  const int64_t* als_rows;
  const float* tt_users;
  const float* als_items_t;
  const float* tt_items;
  const float* tt_items_t;
  const void* prepared;
  int64_t als_ld;
  int64_t n_als_rows;
  int64_t tt_ld;
  int64_t als_items_ld;
  int64_t tt_items_ld;
  int64_t tt_items_t_ld;
  int64_t n_items;
  int32_t als_width;
  int32_t tt_width;
  int32_t n_users;
  int32_t dk;
} hrec_hybrid_batch;
size_t hrec_hybrid_exact_items_bytes(int64_t n_items, int dk);
int hrec_hybrid_exact_prepare(const float* als_items_t, int64_t als_ld, int als_width, const float* tt_items,
                              int64_t tt_ld, int tt_width, int64_t n_items, int dk, void* out, void* stream);
/* Workspace (the same dk) carrying phase 1 into phase 2: 16 B per user and
 * 32-item group + the bf16 user operands — 12.8 MB for 256 users x 100k items. */
size_t hrec_hybrid_exact_workspace_bytes(int n_users, int64_t n_items, int dk);
/* Phase 1 + the exact extremes: als_mm / tt_mm [2, n_users] f32 (the
 * hrec_rows_minmax_f32 layout). All-reduce them across item shards, then: */
int hrec_hybrid_exact_minmax(const hrec_hybrid_batch* batch, float* als_mm, float* tt_mm, void* workspace,
                             size_t workspace_bytes, void* stream);
/* the stable top-k (ties -> smaller item; ids + idx_offset) with the (global)
 * extremes; top_k in [1, 8]. */
int hrec_hybrid_exact_topk(const hrec_hybrid_batch* batch, const float* als_mm, const float* tt_mm, int als_wins,
                           int top_k, int64_t idx_offset, int64_t* out_idx, double* out_val, void* workspace,
                           size_t workspace_bytes, void* stream);
/* Both for ONE shard (als_mm / tt_mm are outputs): 3 launches. */
int hrec_hybrid_exact_local(const hrec_hybrid_batch* batch, int als_wins, int top_k, int64_t idx_offset,
                            float* als_mm, float* tt_mm, int64_t* out_idx, double* out_val, void* workspace,
                            size_t workspace_bytes, void* stream);
/* Diagnostics of the last call: out[b] = item groups rescored for user b's
 * exact extremes, out[n_users + b] = for its top-k, out[2 n_users] = 1 when
 * some user rescored every group (int32, device). */
int hrec_hybrid_exact_counts(const void* workspace, int n_users, int64_t n_items, int dk, int32_t* out,
                             void* stream);

/* ---------------------------------------------------------------------
 * Multi-GPU exchange steps (csrc/comm.hip) for hosts without
 * torch.distributed: one process per GPU, RCCL over xGMI (bound with dlopen
 * at hrec_comm_init; a process that already loaded librccl.so.1 — PyTorch —
 * shares that copy). Rank 0 calls hrec_comm_get_unique_id and hands the 128
 * bytes to every rank (the host's own channel); every rank then calls
 * hrec_comm_init (collective). HREC_E_UNSUPPORTED when RCCL is absent.
 *   C1: hrec_allgather of a rank's factor rows after a half-sweep (recv =
 *       world x count elements, rank-major: the replicated matrix);
 *   C2: hrec_allreduce_minmax — mm is [n_rows][2][n_users] f32 (each model's
 *       [min; max] rows, the hrec_rows_minmax_f32 layout, models consecutive),
 *       replaced in place by the minima / maxima over all ranks (one MIN
 *       all-reduce with the maxima negated);
 *   C3: hrec_allgather (dtype 4 = bytes) of the per-shard top-k candidates. */
int hrec_comm_get_unique_id(uint8_t* id_out /* 128 bytes */);
int hrec_comm_init(int rank, int world, const uint8_t* id /* 128 bytes */, void** comm_out);
int hrec_comm_destroy(void* comm);
/* dtype: 0 f32, 1 f64, 2 i32, 3 i64, 4 u8; count = elements per rank. */
int hrec_allgather(void* comm, const void* send, void* recv, size_t count, int dtype, void* stream);
int hrec_allreduce_minmax(void* comm, float* mm, int n_rows, int64_t n_users, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* HREC_H */
