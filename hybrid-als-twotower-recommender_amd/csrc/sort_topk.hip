// Stable descending top-k for top_k above the selection kernels' bound
// (kTopkSelectMax = 1024): a full stable sort of each row on the device.
//
// The reference ranks with Python's sorted(..., reverse=True)[:k] for any k
// (src/hybrid_system.py:108, src/evaluation.py:30-48 via sorted(dict.items())),
// so hrec_topk_f32 / hrec_topk_f64 / hrec_fuse_topk accept every top_k <= n.
// Up to 1024 they run the segment selections of score.hip; beyond, this path:
//   1. keys: value -> 64-bit key whose ascending order is "larger value first,
//      NaN last" (-0.0 folded onto +0.0 so that it ties with 0.0 as Python's
//      comparison does), position -> 32-bit payload;
//   2. a stable LSD radix sort of (key, flat position) over the whole batch
//      (the in-tree sort of csrc/ingest.hip, 32-bit keys: the low key word
//      carrying (high word, position), then the high word carrying the
//      position), then — several rows — a stable sort by row; LSD radix
//      sorts are stable, so equal values keep ascending position = Python's
//      stable order;
//   3. the first k of each row gathered to (index, value).
// HBM-bound integer work (8 + ceil(log2(rows) / 10) passes over 12 B per
// element).
#include "common.h"

namespace hrec {

template <typename T>
__device__ __forceinline__ uint64_t desc_key(T x) {
  const double v = (double)x;  // f32 -> f64 is exact and order-preserving
  if (v != v) return ~0ull;    // NaN last (better() in score.hip)
  const uint64_t bits = (v == 0.0) ? 0ull : (uint64_t)__double_as_longlong(v);
  const uint64_t asc = (bits >> 63) ? ~bits : (bits | 0x8000000000000000ull);  // ascending-order key
  return ~asc;  // descending; never ~0 (asc == 0 would be a NaN pattern)
}

template <typename T>
__global__ __launch_bounds__(256) void sort_keys_kernel(const T* __restrict__ vals, int64_t n_rows, int64_t n,
                                                        int64_t row_stride, uint32_t* __restrict__ k_lo,
                                                        uint32_t* __restrict__ k_hi, uint32_t* __restrict__ pos) {
  const int64_t total = n_rows * n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / n, c = t - r * n;
    const uint64_t k = desc_key(vals[r * row_stride + c]);
    k_lo[t] = (uint32_t)k;
    k_hi[t] = (uint32_t)(k >> 32);
    pos[t] = (uint32_t)t;  // flat position r n + c (< 2^31)
  }
}

// the row of each sorted flat position: the key of the last (row) pass
__global__ __launch_bounds__(256) void row_keys_kernel(const uint32_t* __restrict__ pos, int64_t m, int64_t n,
                                                       uint32_t* __restrict__ row) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < m; t += (int64_t)gridDim.x * blockDim.x)
    row[t] = (uint32_t)(pos[t] / (uint64_t)n);
}

template <typename T>
__global__ __launch_bounds__(256) void sort_gather_kernel(const T* __restrict__ vals, int64_t n_rows, int64_t n,
                                                          int64_t row_stride, const int32_t* __restrict__ pos_sorted,
                                                          int kk, int64_t* __restrict__ out_idx,
                                                          T* __restrict__ out_val) {
  const int64_t total = n_rows * (int64_t)kk;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / kk, j = t - r * kk;
    const int64_t p = (int64_t)(uint32_t)pos_sorted[r * n + j] - r * n;  // flat -> column
    out_idx[t] = p;
    out_val[t] = vals[r * row_stride + p];
  }
}

namespace {
inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
inline unsigned grid_of(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < 65536 ? (b > 0 ? b : 1) : 65536);
}

// the in-tree sort's workspace, then five 32-bit columns (key words, flat
// positions, the sorts' outputs)
struct SortWs {
  size_t sort, c0, c1, c2, c3, c4, total;
  SortWs(int64_t n_rows, int64_t n) {
    const int64_t m = n_rows * n;
    sort = 0;
    c0 = sort + al256(radix_pairs_ws_bytes(m));
    c1 = c0 + al256(4 * (size_t)m);
    c2 = c1 + al256(4 * (size_t)m);
    c3 = c2 + al256(4 * (size_t)m);
    c4 = c3 + al256(4 * (size_t)m);
    total = c4 + al256(4 * (size_t)m) + 256;
  }
};
}  // namespace

bool sort_topk_fits(int64_t n_rows, int64_t n) { return n_rows >= 1 && n >= 1 && n_rows * n < 0x7fffffffll; }

size_t sort_topk_ws_bytes(int64_t n_rows, int64_t n) {
  if (!sort_topk_fits(n_rows, n)) return 256;
  return SortWs(n_rows, n).total;
}

template <typename T>
int sort_topk_rows(const T* vals, int64_t n_rows, int64_t n, int64_t row_stride, int kk, int64_t* out_idx,
                   T* out_val, void* ws, size_t ws_bytes, hipStream_t s) {
  HREC_REQUIRE(sort_topk_fits(n_rows, n), "topk (sort path): rows * n must be below 2^31");
  HREC_REQUIRE(kk >= 1 && kk <= n, "topk (sort path): need 1 <= top_k <= n");
  const SortWs L(n_rows, n);
  HREC_REQUIRE(ws && ws_bytes >= L.total, "topk (sort path): workspace %zu < %zu bytes", ws_bytes, L.total);
  char* w = static_cast<char*>(ws);
  uint32_t* c0 = reinterpret_cast<uint32_t*>(w + L.c0);
  uint32_t* c1 = reinterpret_cast<uint32_t*>(w + L.c1);
  uint32_t* c2 = reinterpret_cast<uint32_t*>(w + L.c2);
  uint32_t* c3 = reinterpret_cast<uint32_t*>(w + L.c3);
  uint32_t* c4 = reinterpret_cast<uint32_t*>(w + L.c4);
  const int64_t m = n_rows * n;
  // c0 / c1: key words, c2: flat positions
  hipLaunchKernelGGL((sort_keys_kernel<T>), dim3(grid_of(m)), dim3(256), 0, s, vals, n_rows, n, row_stride, c0, c1, c2);
  const uint32_t* ks = nullptr;
  // by the low word carrying (high word, position) -> c3 (high words), c4 (positions)
  int rc = radix_pairs_sort(c0, c1, c2, m, 32, w + L.sort, c3, c4, &ks, s);
  if (rc) return rc;
  // by the high word carrying the position -> c2 (positions sorted by the key)
  rc = radix_pairs_sort(c3, c4, c4, m, 32, w + L.sort, c2, c1, &ks, s);
  if (rc) return rc;
  const int32_t* pos_sorted = reinterpret_cast<const int32_t*>(c2);
  if (n_rows > 1) {  // stable by row: each row's positions keep the key order
    hipLaunchKernelGGL(row_keys_kernel, dim3(grid_of(m)), dim3(256), 0, s, c2, m, n, c0);
    int bits = 1;
    while (bits < 32 && ((int64_t)1 << bits) < n_rows) ++bits;
    rc = radix_pairs_sort(c0, c2, c2, m, bits, w + L.sort, c3, c4, &ks, s);
    if (rc) return rc;
    pos_sorted = reinterpret_cast<const int32_t*>(c3);
  }
  hipLaunchKernelGGL((sort_gather_kernel<T>), dim3(grid_of(n_rows * (int64_t)kk)), dim3(256), 0, s, vals, n_rows, n,
                     row_stride, pos_sorted, kk, out_idx, out_val);
  return check_launch("sort_gather_kernel");
}

template int sort_topk_rows<float>(const float*, int64_t, int64_t, int64_t, int, int64_t*, float*, void*, size_t,
                                   hipStream_t);
template int sort_topk_rows<double>(const double*, int64_t, int64_t, int64_t, int, int64_t*, double*, void*, size_t,
                                    hipStream_t);

}  // namespace hrec
