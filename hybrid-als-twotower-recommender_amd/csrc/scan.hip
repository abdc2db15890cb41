// Prefix sums and extremes of integer columns on the device (the CSR/CSC
// indptr of the synthetic generator, the dense-id ranks of hrec_encode_ids,
// the id range of hrec_minmax_i64): reduce-then-scan over tiles of 4096
// elements — tile sums, one block scans the sums, every tile scans itself
// from its offset. Three streaming passes (read, read + write), any n.
#include "common.h"

namespace hrec {

constexpr int kScanThreads = 256, kScanIPT = 16, kScanTile = kScanThreads * kScanIPT;

inline int64_t scan_tiles(int64_t n) { return (n + kScanTile - 1) / kScanTile; }

size_t scan_ws_bytes(int64_t n) { return (size_t)(scan_tiles(n) > 0 ? scan_tiles(n) : 1) * 8 + 256; }

// inclusive wave scan (64 lanes)
template <typename T>
__device__ __forceinline__ T scan_wave(T x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const T y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  return x;
}

// exclusive block scan of one value per thread; *total = the block's sum
template <typename T, int NT>
__device__ __forceinline__ T scan_block_excl(T x, T* total) {
  __shared__ T wsum[NT / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const T inc = scan_wave(x);
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  T base = 0, tot = 0;
#pragma unroll
  for (int q = 0; q < NT / 64; ++q) {
    if (q < w) base += wsum[q];
    tot += wsum[q];
  }
  __syncthreads();  // wsum is reused by the next call
  *total = tot;
  return base + inc - x;
}

template <typename T>
__global__ __launch_bounds__(kScanThreads) void scan_tile_sum_kernel(const T* __restrict__ in, int64_t n,
                                                                     T* __restrict__ sums) {
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  T a = 0;
#pragma unroll
  for (int e = 0; e < kScanIPT; ++e) {
    const int64_t i = base + (int64_t)e * kScanThreads + threadIdx.x;  // coalesced: order does not matter here
    if (i < n) a += in[i];
  }
  T tot;
  (void)scan_block_excl<T, kScanThreads>(a, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// exclusive scan of the tile sums in place (one block, any count)
template <typename T>
__global__ __launch_bounds__(1024) void scan_sums_kernel(T* __restrict__ sums, int64_t n_tiles) {
  T carry = 0;
  for (int64_t t0 = 0; t0 < n_tiles; t0 += 1024) {
    const int64_t t = t0 + threadIdx.x;
    const T v = t < n_tiles ? sums[t] : (T)0;
    T tot;
    const T ex = scan_block_excl<T, 1024>(v, &tot);
    if (t < n_tiles) sums[t] = carry + ex;
    carry += tot;
  }
}

// out[i] = offset of the tile + the tile's prefix (inclusive or exclusive):
// each thread scans 16 consecutive elements it stages through LDS (coalesced
// loads and stores)
template <typename T, bool EXCL>
__global__ __launch_bounds__(kScanThreads) void scan_tile_kernel(const T* __restrict__ in, int64_t n,
                                                                 const T* __restrict__ offs, T* __restrict__ out) {
  __shared__ T st[kScanTile + kScanTile / 32];  // +1 slot per 32: conflict-free column reads
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  auto slot = [](int q) { return q + (q >> 5); };
#pragma unroll
  for (int e = 0; e < kScanIPT; ++e) {
    const int q = e * kScanThreads + threadIdx.x;
    st[slot(q)] = base + q < n ? in[base + q] : (T)0;
  }
  __syncthreads();
  T v[kScanIPT], a = 0;
#pragma unroll
  for (int e = 0; e < kScanIPT; ++e) {
    v[e] = st[slot(threadIdx.x * kScanIPT + e)];
    a += v[e];
  }
  T tot;
  T run = offs[blockIdx.x] + scan_block_excl<T, kScanThreads>(a, &tot);
#pragma unroll
  for (int e = 0; e < kScanIPT; ++e) {
    const T x = v[e];
    if (!EXCL) run += x;
    st[slot(threadIdx.x * kScanIPT + e)] = run;
    if (EXCL) run += x;
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kScanIPT; ++e) {
    const int q = e * kScanThreads + threadIdx.x;
    if (base + q < n) out[base + q] = st[slot(q)];
  }
}

template <typename T>
int scan_run(const T* in, T* out, int64_t n, bool exclusive, void* ws, hipStream_t s) {
  if (n <= 0) return HREC_OK;
  const int64_t nt = scan_tiles(n);
  T* sums = static_cast<T*>(ws);
  hipLaunchKernelGGL(scan_tile_sum_kernel<T>, dim3((unsigned)nt), dim3(kScanThreads), 0, s, in, n, sums);
  hipLaunchKernelGGL(scan_sums_kernel<T>, dim3(1), dim3(1024), 0, s, sums, nt);
  if (exclusive)
    hipLaunchKernelGGL((scan_tile_kernel<T, true>), dim3((unsigned)nt), dim3(kScanThreads), 0, s, in, n, sums, out);
  else
    hipLaunchKernelGGL((scan_tile_kernel<T, false>), dim3((unsigned)nt), dim3(kScanThreads), 0, s, in, n, sums, out);
  return check_launch("scan");
}

template int scan_run<int32_t>(const int32_t*, int32_t*, int64_t, bool, void*, hipStream_t);
template int scan_run<int64_t>(const int64_t*, int64_t*, int64_t, bool, void*, hipStream_t);

// ---------------------------------------------------------------- extremes
// out[0] = min, out[1] = max of x[0 .. n): per-block extremes, then one
// 64-bit device atomic per block on a slot the first kernel initialised.
__global__ void minmax_init_kernel(int64_t* __restrict__ out) {
  out[0] = INT64_MAX;
  out[1] = INT64_MIN;
}

__global__ __launch_bounds__(256) void minmax_i64_kernel(const int64_t* __restrict__ x, int64_t n,
                                                         int64_t* __restrict__ out) {
  __shared__ int64_t smn[4], smx[4];
  int64_t mn = INT64_MAX, mx = INT64_MIN;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t v = x[i];
    mn = v < mn ? v : mn;
    mx = v > mx ? v : mx;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const int64_t a = __shfl_xor(mn, off, 64), b = __shfl_xor(mx, off, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    smn[w] = mn;
    smx[w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < 4; ++q) {
      mn = smn[q] < mn ? smn[q] : mn;
      mx = smx[q] > mx ? smx[q] : mx;
    }
    atomicMin((long long*)&out[0], (long long)mn);
    atomicMax((long long*)&out[1], (long long)mx);
  }
}

int minmax_i64_run(const int64_t* x, int64_t n, int64_t* out, hipStream_t s) {
  int64_t blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(minmax_init_kernel, dim3(1), dim3(1), 0, s, out);
  hipLaunchKernelGGL(minmax_i64_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, n, out);
  return check_launch("minmax_i64_kernel");
}

}  // namespace hrec
