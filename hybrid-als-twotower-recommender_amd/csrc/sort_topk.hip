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
//   2. an LSD radix sort of (key, position) per row — LSD radix sorts are
//      stable, so equal values keep ascending position = Python's stable order;
//   3. the first k of each row gathered to (index, value).
// HBM-bound integer work (8 passes of 8 bits over 12 B per element).
#include <hipcub/hipcub.hpp>

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
                                                        int64_t row_stride, uint64_t* __restrict__ keys,
                                                        int32_t* __restrict__ pos) {
  const int64_t total = n_rows * n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / n, c = t - r * n;
    keys[t] = desc_key(vals[r * row_stride + c]);
    pos[t] = (int32_t)c;
  }
}

__global__ __launch_bounds__(256) void row_offsets_kernel(int64_t n_rows, int64_t n, int32_t* __restrict__ off) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r <= n_rows) off[r] = (int32_t)(r * n);
}

template <typename T>
__global__ __launch_bounds__(256) void sort_gather_kernel(const T* __restrict__ vals, int64_t n_rows, int64_t n,
                                                          int64_t row_stride, const int32_t* __restrict__ pos_sorted,
                                                          int kk, int64_t* __restrict__ out_idx,
                                                          T* __restrict__ out_val) {
  const int64_t total = n_rows * (int64_t)kk;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / kk, j = t - r * kk;
    const int32_t p = pos_sorted[r * n + j];
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

struct SortWs {
  size_t keys, keys2, pos, pos2, off, temp, total;
  SortWs(int64_t n_rows, int64_t n) {
    const int64_t m = n_rows * n;
    size_t tmp = 0;
    (void)hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, tmp, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                      (const int32_t*)nullptr, (int32_t*)nullptr, (int)m,
                                                      (int)n_rows, (const int32_t*)nullptr, (const int32_t*)nullptr);
    keys = 0;
    keys2 = keys + al256(8 * (size_t)m);
    pos = keys2 + al256(8 * (size_t)m);
    pos2 = pos + al256(4 * (size_t)m);
    off = pos2 + al256(4 * (size_t)m);
    temp = off + al256(4 * (size_t)(n_rows + 1));
    total = temp + al256(tmp) + 256;
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
  uint64_t* keys = reinterpret_cast<uint64_t*>(w + L.keys);
  uint64_t* keys2 = reinterpret_cast<uint64_t*>(w + L.keys2);
  int32_t* pos = reinterpret_cast<int32_t*>(w + L.pos);
  int32_t* pos2 = reinterpret_cast<int32_t*>(w + L.pos2);
  int32_t* off = reinterpret_cast<int32_t*>(w + L.off);
  const int64_t m = n_rows * n;
  hipLaunchKernelGGL((sort_keys_kernel<T>), dim3(grid_of(m)), dim3(256), 0, s, vals, n_rows, n, row_stride, keys, pos);
  hipLaunchKernelGGL(row_offsets_kernel, dim3(grid_of(n_rows + 1)), dim3(256), 0, s, n_rows, n, off);
  size_t tb = L.total - L.temp;
  if (hipcub::DeviceSegmentedRadixSort::SortPairs(w + L.temp, tb, keys, keys2, pos, pos2, (int)m, (int)n_rows, off,
                                                  off + 1, 0, 64, s) != hipSuccess)
    return check_launch("topk (sort path): radix sort");
  hipLaunchKernelGGL((sort_gather_kernel<T>), dim3(grid_of(n_rows * (int64_t)kk)), dim3(256), 0, s, vals, n_rows, n,
                     row_stride, pos2, kk, out_idx, out_val);
  return check_launch("sort_gather_kernel");
}

template int sort_topk_rows<float>(const float*, int64_t, int64_t, int64_t, int, int64_t*, float*, void*, size_t,
                                   hipStream_t);
template int sort_topk_rows<double>(const double*, int64_t, int64_t, int64_t, int, int64_t*, double*, void*, size_t,
                                    hipStream_t);

}  // namespace hrec
