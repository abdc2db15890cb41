// Ingest: ratings as COO columns -> the CSR / CSC the
// half-sweep consumes, on the device.
//
// Replaces the reference's hand-over of a pandas DataFrame to Spark
// (src/als_model.py:51-62: createDataFrame + ALS.fit, which keys factors by the
// integer user / item ids and keeps duplicate (user, item) ratings as separate
// terms of the normal equations). Two steps:
//   hrec_encode_ids  : int64 ids -> sorted distinct ids + a dense int32 code per
//                      entry (numpy.unique(ids, return_inverse=True)); with the
//                      id range [lo, hi] known (hrec_minmax_i64) a range below
//                      2^31 sorts 32-bit keys on only the bits it spans;
//   hrec_coo_to_csr  : (row code, col code, rating) -> indptr / indices / values,
//                      rows ascending, entries of a row in input order
//                      (numpy.argsort(rows, kind="stable")).
// Both are radix sorts (hipCUB, stable LSD) plus O(n) integer passes; HBM-bound.
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace hrec {

__global__ __launch_bounds__(256) void iota_i32_kernel(int32_t* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (int32_t)i;
}

// keys32[i] = ids[i] - lo (caller guarantees lo <= ids <= hi, hi - lo < 2^31)
__global__ __launch_bounds__(256) void shift_keys_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t lo,
                                                         int32_t* __restrict__ keys32) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    keys32[i] = (int32_t)(ids[i] - lo);
}

// flag[i] = 1 where sorted key i starts a new distinct value
template <typename K>
__global__ __launch_bounds__(256) void distinct_flags_kernel(const K* __restrict__ keys, int64_t n,
                                                             int32_t* __restrict__ flag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    flag[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}

// codes[pos[i]] = rank of sorted key i among the distinct keys; the first
// occurrence of each distinct key writes it (+ lo) to uniq; the last thread
// writes the distinct count.
template <typename K>
__global__ __launch_bounds__(256) void scatter_codes_kernel(const K* __restrict__ keys, int64_t lo,
                                                            const int32_t* __restrict__ pos,
                                                            const int32_t* __restrict__ flag,
                                                            const int32_t* __restrict__ incl, int64_t n,
                                                            int32_t* __restrict__ codes, int64_t* __restrict__ uniq,
                                                            int64_t* __restrict__ n_uniq) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t c = incl[i] - 1;
    codes[pos[i]] = c;
    if (flag[i]) uniq[c] = (int64_t)keys[i] + lo;
    if (i == n - 1) *n_uniq = (int64_t)incl[i];
  }
}

// Dense id ranges (span <= n): np.unique(return_inverse) without a sort.
// Mark the ids present in a span-long table, one inclusive scan gives every
// present id its rank among the sorted distinct ids, and the codes are read
// back from the table: two streaming passes over the ids instead of a radix
// sort of (id, position) pairs. Same codes and uniq as the sort path.
__global__ __launch_bounds__(256) void mark_present_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t lo,
                                                           int64_t span, int32_t* __restrict__ present) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = ids[i] - lo;
    if (v >= 0 && v < span) present[v] = 1;  // every writer stores the same value
  }
}

__global__ __launch_bounds__(256) void codes_from_rank_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t lo,
                                                              int64_t span, const int32_t* __restrict__ incl,
                                                              int32_t* __restrict__ codes) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = ids[i] - lo;
    codes[i] = (v >= 0 && v < span) ? incl[v] - 1 : -1;  // out-of-range ids (a caller error) -> -1
  }
}

__global__ __launch_bounds__(256) void uniq_from_rank_kernel(const int32_t* __restrict__ present,
                                                             const int32_t* __restrict__ incl, int64_t span,
                                                             int64_t lo, int64_t* __restrict__ uniq,
                                                             int64_t* __restrict__ n_uniq) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < span; v += (int64_t)gridDim.x * blockDim.x) {
    if (present[v]) uniq[incl[v] - 1] = v + lo;
    if (v == span - 1) *n_uniq = (int64_t)incl[v];
  }
}

__global__ void minmax_store_kernel(const int64_t* __restrict__ mn, const int64_t* __restrict__ mx,
                                    int64_t* __restrict__ out) {
  out[0] = *mn;
  out[1] = *mx;
}

// indptr from row-sorted keys: indptr[r] = first i with keys[i] >= r.
// Each boundary between distinct keys fills the empty rows in between.
__global__ __launch_bounds__(256) void indptr_from_sorted_kernel(const int32_t* __restrict__ keys, int64_t nnz,
                                                                 int64_t n_rows, int64_t* __restrict__ indptr) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= nnz; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t lo = (i == 0) ? -1 : (int64_t)keys[i - 1];
    const int64_t hi = (i == nnz) ? n_rows : (int64_t)keys[i];
    for (int64_t r = lo + 1; r <= hi && r <= n_rows; ++r) indptr[r] = i;
  }
}

// (col, rating bits) packed in one 64-bit radix-sort value: the sort then
// carries the entries along (no random gather after it)
__global__ __launch_bounds__(256) void pack_entries_kernel(const int32_t* __restrict__ cols,
                                                           const float* __restrict__ vals, int64_t nnz,
                                                           uint64_t* __restrict__ packed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * blockDim.x)
    packed[i] = (uint64_t)(uint32_t)cols[i] | ((uint64_t)__float_as_uint(vals[i]) << 32);
}

__global__ __launch_bounds__(256) void unpack_entries_kernel(const uint64_t* __restrict__ packed, int64_t nnz,
                                                             int32_t* __restrict__ indices,
                                                             float* __restrict__ values) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t v = packed[i];
    indices[i] = (int32_t)(uint32_t)v;
    values[i] = __uint_as_float((uint32_t)(v >> 32));
  }
}

// *flag = 1 if some x[i] > x[i + 1] (the caller zeroes it first)
__global__ __launch_bounds__(256) void descent_kernel(const int32_t* __restrict__ x, int64_t n, int32_t* __restrict__ flag) {
  bool d = false;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += (int64_t)gridDim.x * blockDim.x)
    d |= x[i] > x[i + 1];
  if (__any(d) && (threadIdx.x & 63) == 0) *flag = 1;
}

// rows already non-decreasing: the CSR is the input order (the stable sort is the identity)
__global__ __launch_bounds__(256) void copy_entries_kernel(const int32_t* __restrict__ cols, const float* __restrict__ vals,
                                                           int64_t nnz, int32_t* __restrict__ indices,
                                                           float* __restrict__ values) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * blockDim.x) {
    indices[i] = cols[i];
    values[i] = vals[i];
  }
}

inline unsigned grid_for(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < 65536 ? (b > 0 ? b : 1) : 65536);
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

int bits_for(int64_t n_rows) {  // radix bits covering codes 0 .. n_rows-1
  int b = 1;
  while (b < 32 && ((int64_t)1 << b) < n_rows) ++b;
  return b;
}

// Workspace layout of hrec_encode_ids (all 256-B aligned). keys holds the
// sorted 64-bit keys, or the shifted 32-bit keys and their sorted copy.
struct EncodeWs {
  size_t keys, pos, pos2, flag, incl, temp, total;
  explicit EncodeWs(int64_t n) {
    size_t sort_tmp = 0, sort32_tmp = 0, scan_tmp = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (const int64_t*)nullptr, (int64_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort32_tmp, (const int32_t*)nullptr, (int32_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, scan_tmp, (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
    if (sort32_tmp > sort_tmp) sort_tmp = sort32_tmp;
    keys = 0;
    pos = keys + align256(8 * (size_t)n);
    pos2 = pos + align256(4 * (size_t)n);
    flag = pos2 + align256(4 * (size_t)n);
    incl = flag + align256(4 * (size_t)n);
    temp = incl + align256(4 * (size_t)n);
    total = temp + align256(sort_tmp > scan_tmp ? sort_tmp : scan_tmp);
  }
};

// keys: sorted row codes; pk / pk2: packed (col, rating) entries before /
// after the sort (8 B each)
struct CsrWs {
  size_t keys, pk, pk2, temp, total;
  CsrWs(int64_t nnz, int bits) {
    size_t sort_tmp = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (const int32_t*)nullptr, (int32_t*)nullptr,
                                             (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)nnz, 0, bits);
    keys = 0;
    pk = keys + align256(4 * (size_t)nnz);
    pk2 = pk + align256(8 * (size_t)nnz);
    temp = pk2 + align256(8 * (size_t)nnz);
    total = temp + align256(sort_tmp);
  }
};

}  // namespace hrec

using namespace hrec;

extern "C" size_t hrec_encode_ids_workspace_bytes(int64_t n) {
  if (n <= 0 || n >= 0x7fffffffll) return 0;
  return EncodeWs(n).total;
}

extern "C" int hrec_encode_ids(const int64_t* ids, int64_t n, int64_t id_lo, int64_t id_hi, int64_t* uniq,
                               int64_t* n_uniq, int32_t* codes, void* ws, size_t ws_bytes, void* stream) {
  HREC_REQUIRE(n >= 0 && n < 0x7fffffffll, "encode_ids: n=%lld out of range [0, 2^31-1)", (long long)n);
  HREC_REQUIRE(n_uniq, "encode_ids: null n_uniq");
  HREC_REQUIRE(id_lo <= id_hi, "encode_ids: id_lo > id_hi");
  hipStream_t s = as_stream(stream);
  if (n == 0) {
    if (hipMemsetAsync(n_uniq, 0, sizeof(int64_t), s) != hipSuccess) return check_launch("encode_ids: memset");
    return HREC_OK;
  }
  HREC_REQUIRE(ids && uniq && codes && ws, "encode_ids: null pointer");
  const EncodeWs L(n);
  HREC_REQUIRE(ws_bytes >= L.total, "encode_ids: workspace %zu < %zu bytes", ws_bytes, L.total);
  char* w = static_cast<char*>(ws);
  int32_t* pos = reinterpret_cast<int32_t*>(w + L.pos);
  int32_t* pos2 = reinterpret_cast<int32_t*>(w + L.pos2);
  int32_t* flag = reinterpret_cast<int32_t*>(w + L.flag);
  int32_t* incl = reinterpret_cast<int32_t*>(w + L.incl);
  void* temp = w + L.temp;
  size_t temp_bytes = L.total - L.temp;
  const unsigned g = grid_for(n);
  // A narrow id range sorts (id - lo) on only the bits it spans.
  const bool narrow = (uint64_t)id_hi - (uint64_t)id_lo < 0x7fffffffull;
  const int64_t span = narrow ? (int64_t)((uint64_t)id_hi - (uint64_t)id_lo) + 1 : 0;
  if (narrow && span <= n && span < 0x7fffffffll) {
    // dense range: the span-long tables fit the flag / incl buffers (n entries each)
    if (hipMemsetAsync(flag, 0, (size_t)span * sizeof(int32_t), s) != hipSuccess)
      return check_launch("encode_ids: memset");
    hipLaunchKernelGGL(mark_present_kernel, dim3(g), dim3(256), 0, s, ids, n, id_lo, span, flag);
    if (hipcub::DeviceScan::InclusiveSum(temp, temp_bytes, flag, incl, (int)span, s) != hipSuccess)
      return check_launch("encode_ids: scan");
    hipLaunchKernelGGL(codes_from_rank_kernel, dim3(g), dim3(256), 0, s, ids, n, id_lo, span, incl, codes);
    hipLaunchKernelGGL(uniq_from_rank_kernel, dim3(grid_for(span)), dim3(256), 0, s, flag, incl, span, id_lo, uniq,
                       n_uniq);
    return check_launch("encode_ids: dense");
  }
  hipLaunchKernelGGL(iota_i32_kernel, dim3(g), dim3(256), 0, s, pos, n);
  if (narrow) {
    int32_t* k32 = reinterpret_cast<int32_t*>(w + L.keys);
    int32_t* k32s = k32 + n;
    const int bits = bits_for((int64_t)((uint64_t)id_hi - (uint64_t)id_lo) + 1);
    hipLaunchKernelGGL(shift_keys_kernel, dim3(g), dim3(256), 0, s, ids, n, id_lo, k32);
    if (hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k32, k32s, pos, pos2, (int)n, 0, bits, s) != hipSuccess)
      return check_launch("encode_ids: radix sort");
    hipLaunchKernelGGL(distinct_flags_kernel<int32_t>, dim3(g), dim3(256), 0, s, k32s, n, flag);
    temp_bytes = L.total - L.temp;
    if (hipcub::DeviceScan::InclusiveSum(temp, temp_bytes, flag, incl, (int)n, s) != hipSuccess)
      return check_launch("encode_ids: scan");
    hipLaunchKernelGGL(scatter_codes_kernel<int32_t>, dim3(g), dim3(256), 0, s, k32s, id_lo, pos2, flag, incl, n,
                       codes, uniq, n_uniq);
  } else {
    int64_t* keys = reinterpret_cast<int64_t*>(w + L.keys);
    if (hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, ids, keys, pos, pos2, (int)n, 0, 64, s) != hipSuccess)
      return check_launch("encode_ids: radix sort");
    hipLaunchKernelGGL(distinct_flags_kernel<int64_t>, dim3(g), dim3(256), 0, s, keys, n, flag);
    temp_bytes = L.total - L.temp;
    if (hipcub::DeviceScan::InclusiveSum(temp, temp_bytes, flag, incl, (int)n, s) != hipSuccess)
      return check_launch("encode_ids: scan");
    hipLaunchKernelGGL(scatter_codes_kernel<int64_t>, dim3(g), dim3(256), 0, s, keys, (int64_t)0, pos2, flag, incl,
                       n, codes, uniq, n_uniq);
  }
  return check_launch("encode_ids");
}

extern "C" size_t hrec_minmax_i64_workspace_bytes(int64_t n) {
  if (n <= 0 || n >= 0x7fffffffll) return 0;
  size_t a = 0, b = 0;
  (void)hipcub::DeviceReduce::Min(nullptr, a, (const int64_t*)nullptr, (int64_t*)nullptr, (int)n);
  (void)hipcub::DeviceReduce::Max(nullptr, b, (const int64_t*)nullptr, (int64_t*)nullptr, (int)n);
  return 512 + align256(a > b ? a : b);
}

extern "C" int hrec_minmax_i64(const int64_t* x, int64_t n, int64_t* out, void* ws, size_t ws_bytes,
                               void* stream) {
  HREC_REQUIRE(n > 0 && n < 0x7fffffffll, "minmax_i64: n=%lld out of range [1, 2^31-1)", (long long)n);
  HREC_REQUIRE(x && out && ws, "minmax_i64: null pointer");
  const size_t need = hrec_minmax_i64_workspace_bytes(n);
  HREC_REQUIRE(ws_bytes >= need, "minmax_i64: workspace %zu < %zu bytes", ws_bytes, need);
  hipStream_t s = as_stream(stream);
  char* w = static_cast<char*>(ws);
  int64_t* mn = reinterpret_cast<int64_t*>(w);
  int64_t* mx = reinterpret_cast<int64_t*>(w + 256);
  size_t tb = need - 512;
  if (hipcub::DeviceReduce::Min(w + 512, tb, x, mn, (int)n, s) != hipSuccess) return check_launch("minmax_i64: min");
  tb = need - 512;
  if (hipcub::DeviceReduce::Max(w + 512, tb, x, mx, (int)n, s) != hipSuccess) return check_launch("minmax_i64: max");
  hipLaunchKernelGGL(minmax_store_kernel, dim3(1), dim3(1), 0, s, mn, mx, out);
  return check_launch("minmax_i64");
}

extern "C" size_t hrec_coo_to_csr_workspace_bytes(int64_t nnz, int64_t n_rows) {
  if (nnz <= 0 || nnz >= 0x7fffffffll || n_rows <= 0 || n_rows >= 0x7fffffffll) return 0;
  return CsrWs(nnz, bits_for(n_rows)).total;
}

extern "C" int hrec_coo_to_csr(const int32_t* rows, const int32_t* cols, const float* vals, int64_t nnz,
                               int64_t n_rows, int64_t* indptr, int32_t* indices, float* values, void* ws,
                               size_t ws_bytes, void* stream) {
  HREC_REQUIRE(nnz >= 0 && nnz < 0x7fffffffll, "coo_to_csr: nnz=%lld out of range", (long long)nnz);
  HREC_REQUIRE(n_rows >= 0 && n_rows < 0x7fffffffll, "coo_to_csr: n_rows=%lld out of range", (long long)n_rows);
  HREC_REQUIRE(indptr, "coo_to_csr: null indptr");
  hipStream_t s = as_stream(stream);
  if (nnz == 0) {
    if (hipMemsetAsync(indptr, 0, sizeof(int64_t) * (size_t)(n_rows + 1), s) != hipSuccess)
      return check_launch("coo_to_csr: memset");
    return HREC_OK;
  }
  HREC_REQUIRE(n_rows > 0, "coo_to_csr: entries but no rows");
  HREC_REQUIRE(rows && cols && vals && indices && values && ws, "coo_to_csr: null pointer");
  const int bits = bits_for(n_rows);
  const CsrWs L(nnz, bits);
  HREC_REQUIRE(ws_bytes >= L.total, "coo_to_csr: workspace %zu < %zu bytes", ws_bytes, L.total);
  char* w = static_cast<char*>(ws);
  int32_t* keys = reinterpret_cast<int32_t*>(w + L.keys);
  uint64_t* pk = reinterpret_cast<uint64_t*>(w + L.pk);
  uint64_t* pk2 = reinterpret_cast<uint64_t*>(w + L.pk2);
  size_t temp_bytes = L.total - L.temp;
  hipLaunchKernelGGL(pack_entries_kernel, dim3(grid_for(nnz)), dim3(256), 0, s, cols, vals, nnz, pk);
  if (hipcub::DeviceRadixSort::SortPairs(w + L.temp, temp_bytes, rows, keys, pk, pk2, (int)nnz, 0, bits, s) !=
      hipSuccess)
    return check_launch("coo_to_csr: radix sort");
  hipLaunchKernelGGL(unpack_entries_kernel, dim3(grid_for(nnz)), dim3(256), 0, s, pk2, nnz, indices, values);
  hipLaunchKernelGGL(indptr_from_sorted_kernel, dim3(grid_for(nnz + 1)), dim3(256), 0, s, keys, nnz, n_rows,
                     indptr);
  return check_launch("coo_to_csr");
}

extern "C" int hrec_rows_descending_pairs(const int32_t* rows, int64_t n, int32_t* out, void* stream) {
  HREC_REQUIRE(n >= 0 && out, "rows_descending_pairs: bad argument");
  hipStream_t s = as_stream(stream);
  if (hipMemsetAsync(out, 0, sizeof(int32_t), s) != hipSuccess) return check_launch("rows_descending_pairs: memset");
  if (n < 2) return HREC_OK;
  HREC_REQUIRE(rows, "rows_descending_pairs: null rows");
  hipLaunchKernelGGL(descent_kernel, dim3(grid_for(n)), dim3(256), 0, s, rows, n, out);
  return check_launch("descent_kernel");
}

extern "C" int hrec_coo_to_csr_sorted(const int32_t* rows, const int32_t* cols, const float* vals, int64_t nnz,
                                      int64_t n_rows, int64_t* indptr, int32_t* indices, float* values,
                                      void* stream) {
  HREC_REQUIRE(nnz >= 0 && nnz < 0x7fffffffll && n_rows >= 0 && n_rows < 0x7fffffffll,
               "coo_to_csr_sorted: bad shape");
  HREC_REQUIRE(indptr, "coo_to_csr_sorted: null indptr");
  hipStream_t s = as_stream(stream);
  if (nnz == 0) {
    if (hipMemsetAsync(indptr, 0, sizeof(int64_t) * (size_t)(n_rows + 1), s) != hipSuccess)
      return check_launch("coo_to_csr_sorted: memset");
    return HREC_OK;
  }
  HREC_REQUIRE(n_rows > 0 && rows && cols && vals && indices && values, "coo_to_csr_sorted: null pointer");
  hipLaunchKernelGGL(copy_entries_kernel, dim3(grid_for(nnz)), dim3(256), 0, s, cols, vals, nnz, indices, values);
  hipLaunchKernelGGL(indptr_from_sorted_kernel, dim3(grid_for(nnz + 1)), dim3(256), 0, s, rows, nnz, n_rows, indptr);
  return check_launch("coo_to_csr_sorted");
}

// ------------------------------------------------------- shard layouts
// x[i] = table[x[i]] in place (the CSR/CSC column ids of an nnz-balanced
// ALS shard -> rows of the padded replicated factor buffer,
// src/als_engine.py:RowLayout). Ids outside [0, table_n) become -1 (the
// half-sweep's structured loads read those as zero rows).
namespace hrec {
__global__ __launch_bounds__(256) void remap_i32_kernel(int32_t* __restrict__ x, int64_t n,
                                                        const int32_t* __restrict__ table, int64_t table_n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int32_t v = x[i];
    x[i] = (v >= 0 && v < table_n) ? table[v] : -1;
  }
}
}  // namespace hrec

extern "C" int hrec_remap_i32(int32_t* x, int64_t n, const int32_t* table, int64_t table_n, void* stream) {
  HREC_REQUIRE(n >= 0 && table_n >= 0, "remap_i32: bad shape");
  if (n == 0) return HREC_OK;
  HREC_REQUIRE(x && table, "remap_i32: null pointer");
  int64_t grid = (n + 255) / 256;
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(remap_i32_kernel, dim3((unsigned)grid), dim3(256), 0, as_stream(stream), x, n, table, table_n);
  return check_launch("remap_i32_kernel");
}
