// K10: the ALS cold-start fallback of every catalogue item, once per model
// ("GEMM + top-k, precomputed once").
//
// ALSModel.predict_for_user (src/als_model.py:78-86) gives an item the
// transform left NaN (an unknown user or item, Spark's coldStartStrategy) the
// mean 'rating' of the <= 3 items most similar to it (_find_similar_items,
// :93-104: sklearn cosine_similarity of the item's feature vector with every
// OTHER item's, sorted(..., reverse=True)[:3], kept when sim > 0.5), else the
// global mean. That value depends on the item alone, not on the user, so it
// is a per-model vector: computed here for all n items in one pass instead of
// one cosine row per NaN item per call (every test user of the
// reference's protocol is cold, so every candidate takes the fallback).
//
//   1. cold_norm_kernel: x_j = f_j / |f_j| (a zero norm -> 1), the
//      arithmetic of cosine_kernel (csrc/score.hip) and of sklearn's
//      normalize: the same bits for every similarity;
//   2. cold_pairs_kernel: a thread per query item q, a block per (256
//      queries, item slice); the slice's rows staged in LDS (every thread reads
//      the same row: a broadcast), sim(q, j) = sum_c x_qc x_jc as the
//      sequential non-FMA f64 chain of cosine_kernel; the query keeps the 3
//      best (value, then smaller j) of the items j != q with sim > 0.5 — the
//      top 3 of all items filtered by sim > 0.5 is exactly the top 3 of those
//      above 0.5 (they rank above every other item), so nothing else is kept;
//   3. cold_merge_kernel: per query the slices' lists merged in slice order
//      (j ascending: an equal value from a later slice ranks after), then the
//      mean of the kept ratings as np.mean sums a short list: ((r0 + r1) + r2)
//      / count, in rank order.
// Work: n^2 (2 dim + 1) f64 operations, no HBM traffic beyond the n x dim
// features per slice (L2-resident): VALU-bound (0.1 s at 10^6 items).
#include "common.h"

namespace hrec {

constexpr int kColdQ = 256;     // queries per block (one per thread)
constexpr int kColdTile = 256;  // items staged per LDS round
constexpr int kColdMaxDim = 16;
constexpr int kColdK = 3;       // _find_similar_items' k

__global__ __launch_bounds__(256) void cold_norm_kernel(const double* __restrict__ feats, int64_t n, int dim,
                                                        double* __restrict__ x) {
#pragma clang fp contract(off)
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const double* f = feats + j * dim;
  double nr = 0.0;
  for (int c = 0; c < dim; ++c) nr = nr + f[c] * f[c];
  nr = sqrt(nr);
  if (nr == 0.0) nr = 1.0;
  for (int c = 0; c < dim; ++c) x[j * dim + c] = f[c] / nr;
}

struct ColdTop {
  double v[kColdK];
  int j[kColdK];
  int n;
};

// insert (val, j) into a list ranked by value, ties by smaller j; every
// candidate arrives with a larger j than the entries already there
__device__ __forceinline__ void cold_insert(ColdTop& t, double val, int j) {
  if (t.n == kColdK && !(val > t.v[kColdK - 1])) return;
  int p = t.n < kColdK ? t.n : kColdK - 1;
  while (p > 0 && val > t.v[p - 1]) {
    t.v[p] = t.v[p - 1];
    t.j[p] = t.j[p - 1];
    --p;
  }
  t.v[p] = val;
  t.j[p] = j;
  if (t.n < kColdK) ++t.n;
}

template <int MAXD>
__global__ __launch_bounds__(kColdQ) void cold_pairs_kernel(const double* __restrict__ x, int64_t n, int dim,
                                                            int64_t slice, double* __restrict__ pv,
                                                            int* __restrict__ pj, int* __restrict__ pn) {
#pragma clang fp contract(off)
  __shared__ double xs[kColdTile * MAXD];
  const int64_t q = (int64_t)blockIdx.x * kColdQ + threadIdx.x;
  const int s = blockIdx.y;
  const int64_t j0 = (int64_t)s * slice;
  const int64_t j1 = j0 + slice < n ? j0 + slice : n;
  double xq[MAXD];
#pragma unroll
  for (int c = 0; c < MAXD; ++c) xq[c] = (q < n && c < dim) ? x[q * dim + c] : 0.0;
  ColdTop t;
  t.n = 0;
  for (int64_t b = j0; b < j1; b += kColdTile) {
    const int m = (int)(j1 - b < kColdTile ? j1 - b : kColdTile);
    __syncthreads();
    for (int o = threadIdx.x; o < m * dim; o += kColdQ) xs[(o / dim) * MAXD + o % dim] = x[b * dim + o];
    __syncthreads();
    if (q < n) {
      for (int r = 0; r < m; ++r) {
        const double* xr = xs + r * MAXD;
        double dot = 0.0;
#pragma unroll
        for (int c = 0; c < MAXD; ++c)
          if (c < dim) dot = dot + xq[c] * xr[c];
        const int j = (int)(b + r);
        if (dot > 0.5 && j != q) cold_insert(t, dot, j);
      }
    }
  }
  if (q >= n) return;
  const int64_t o = (q * gridDim.y + s) * kColdK;
  for (int e = 0; e < kColdK; ++e) {
    pv[o + e] = e < t.n ? t.v[e] : 0.0;
    pj[o + e] = e < t.n ? t.j[e] : -1;
  }
  pn[q * gridDim.y + s] = t.n;
}

__global__ __launch_bounds__(256) void cold_merge_kernel(const double* __restrict__ pv, const int* __restrict__ pj,
                                                         const int* __restrict__ pn, int64_t n, int n_slices,
                                                         const double* __restrict__ ratings,
                                                         double* __restrict__ out_mean, int* __restrict__ out_count,
                                                         int* __restrict__ out_idx) {
#pragma clang fp contract(off)
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= n) return;
  ColdTop t;
  t.n = 0;
  for (int s = 0; s < n_slices; ++s) {
    const int64_t o = (q * n_slices + s) * kColdK;
    const int m = pn[q * n_slices + s];
    for (int e = 0; e < m; ++e) cold_insert(t, pv[o + e], pj[o + e]);
  }
  double sum = 0.0;
  for (int e = 0; e < t.n; ++e) sum = e == 0 ? ratings[t.j[0]] : sum + ratings[t.j[e]];
  out_mean[q] = t.n ? sum / (double)t.n : 0.0;
  out_count[q] = t.n;
  if (out_idx)
    for (int e = 0; e < kColdK; ++e) out_idx[q * kColdK + e] = e < t.n ? t.j[e] : -1;
}

// item slices per query tile: ~2048 blocks over the chip, each slice at
// least one LDS tile
static int cold_slices(int64_t n) {
  const int64_t qt = (n + kColdQ - 1) / kColdQ;
  int64_t s = (2048 + qt - 1) / qt;
  const int64_t tiles = (n + kColdTile - 1) / kColdTile;
  if (s > tiles) s = tiles;
  if (s < 1) s = 1;
  if (s > 65535) s = 65535;
  return (int)s;
}

static size_t cold_al(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace hrec

using namespace hrec;

extern "C" size_t hrec_cold_fallback_workspace_bytes(int64_t n_items, int dim) {
  const int64_t n = n_items > 0 ? n_items : 0;
  const size_t S = (size_t)cold_slices(n);
  return cold_al((size_t)n * (dim > 0 ? dim : 1) * 8) + cold_al((size_t)n * S * kColdK * 8) +
         cold_al((size_t)n * S * kColdK * 4) + cold_al((size_t)n * S * 4) + 256;
}

extern "C" int hrec_cold_fallback(const double* feats, const double* ratings, int64_t n_items, int dim,
                                  double* out_mean, int32_t* out_count, int32_t* out_idx, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  HREC_REQUIRE(n_items >= 0 && n_items < ((int64_t)1 << 31) && dim >= 1 && dim <= kColdMaxDim,
               "cold_fallback: need 0 <= n_items < 2^31 and 1 <= dim <= %d", kColdMaxDim);
  if (n_items == 0) return HREC_OK;
  HREC_REQUIRE(feats && ratings && out_mean && out_count && workspace, "cold_fallback: null pointer");
  const size_t need = hrec_cold_fallback_workspace_bytes(n_items, dim);
  HREC_REQUIRE(workspace_bytes >= need, "cold_fallback: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t s = as_stream(stream);
  const int S = cold_slices(n_items);
  char* p = (char*)workspace;
  double* x = (double*)p;
  p += cold_al((size_t)n_items * dim * 8);
  double* pv = (double*)p;
  p += cold_al((size_t)n_items * S * kColdK * 8);
  int* pj = (int*)p;
  p += cold_al((size_t)n_items * S * kColdK * 4);
  int* pn = (int*)p;
  const unsigned nb = (unsigned)((n_items + 255) / 256);
  hipLaunchKernelGGL(cold_norm_kernel, dim3(nb), dim3(256), 0, s, feats, n_items, dim, x);
  int rc = check_launch("cold_norm_kernel");
  if (rc) return rc;
  const int64_t slice = ((n_items + S - 1) / S + kColdTile - 1) / kColdTile * kColdTile;
  const dim3 grid((unsigned)((n_items + kColdQ - 1) / kColdQ), (unsigned)S);
  if (dim <= 4)
    hipLaunchKernelGGL(cold_pairs_kernel<4>, grid, dim3(kColdQ), 0, s, x, n_items, dim, slice, pv, pj, pn);
  else if (dim <= 8)
    hipLaunchKernelGGL(cold_pairs_kernel<8>, grid, dim3(kColdQ), 0, s, x, n_items, dim, slice, pv, pj, pn);
  else
    hipLaunchKernelGGL(cold_pairs_kernel<16>, grid, dim3(kColdQ), 0, s, x, n_items, dim, slice, pv, pj, pn);
  rc = check_launch("cold_pairs_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(cold_merge_kernel, dim3(nb), dim3(256), 0, s, pv, pj, pn, n_items, S, ratings, out_mean,
                     out_count, out_idx);
  return check_launch("cold_merge_kernel");
}
