// K10: synthetic interaction matrix (CSR / CSC shards) and ALS initial
// factors, generated on the device from counter-based hashes so that any
// shard layout (and the CPU oracle) sees bit-identical data.
#include "common.h"

namespace hrec {

// One wave per output row; the wave sweeps the other dimension 64 columns
// per step. Integer-only: the hash is two 64-bit multiplies.
__global__ __launch_bounds__(256) void synth_count_kernel(uint64_t seed, uint64_t thr,
                                                          int64_t row_begin, int64_t n_rows,
                                                          int64_t n_cols, int transposed,
                                                          int64_t* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= n_rows) return;
  const uint64_t g = (uint64_t)(row_begin + r);
  uint32_t cnt = 0;
  for (int64_t c = lane; c < n_cols; c += kWave) {
    const uint64_t h = transposed ? pair_hash(seed, (uint64_t)c, g) : pair_hash(seed, g, (uint64_t)c);
    cnt += (h < thr) ? 1u : 0u;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, kWave);
  if (lane == 0) counts[r] = (int64_t)cnt;
}

__global__ __launch_bounds__(256) void synth_fill_kernel(uint64_t seed, uint64_t seed2, uint64_t thr,
                                                         int64_t row_begin, int64_t n_rows,
                                                         int64_t n_cols, int transposed, int n_levels,
                                                         const int64_t* __restrict__ indptr,
                                                         int32_t* __restrict__ indices,
                                                         float* __restrict__ values) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= n_rows) return;
  const uint64_t g = (uint64_t)(row_begin + r);
  int64_t pos = indptr[r];
  for (int64_t c0 = 0; c0 < n_cols; c0 += kWave) {
    const int64_t c = c0 + lane;
    bool hit = false;
    uint64_t u = 0, i = 0;
    if (c < n_cols) {
      u = transposed ? (uint64_t)c : g;
      i = transposed ? g : (uint64_t)c;
      hit = pair_hash(seed, u, i) < thr;
    }
    const uint64_t mask = __ballot(hit);
    if (hit) {
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
      indices[pos + below] = (int32_t)c;
      values[pos + below] = (float)(pair_hash(seed2, u, i) % (uint64_t)n_levels);
    }
    pos += __popcll(mask);
  }
}

// Gaussian-like init: z = sum of four 22-bit uniforms - 2 (exact in f32),
// L2-normalised with a sequential f64 sum — bit-reproducible on the host.
__global__ __launch_bounds__(256) void init_factors_kernel(uint64_t seed, int64_t row_begin,
                                                           int64_t n_rows, int k, int kp,
                                                           float* __restrict__ out) {
  __shared__ float z_sh[4][256];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * 4 + w;
  if (r >= n_rows) return;
  const uint64_t g = (uint64_t)(row_begin + r);
  float z[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {  // columns lane, lane + 64, lane + 128, lane + 192
    const int c = lane + 64 * q;
    z[q] = 0.f;
    if (c < k) {
      uint32_t acc = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) acc += (uint32_t)(pair_hash(seed, g, (uint64_t)(c * 4 + t)) >> 42);
      z[q] = (float)acc * (1.0f / 4194304.0f) - 2.0f;
    }
    z_sh[w][c] = z[q];
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  double s = 0.0;
  for (int c = 0; c < k; ++c) {
    const double zc = (double)z_sh[w][c];
    s += zc * zc;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = lane + 64 * q;
    float x = 0.f;
    if (c < k && s > 0.0) x = (float)((double)z[q] * (1.0 / sqrt(s)));
    if (c < kp) out[r * kp + c] = x;
  }
}

}  // namespace hrec

using namespace hrec;

extern "C" int hrec_synth_row_counts(uint64_t seed, uint64_t threshold, int64_t row_begin,
                                     int64_t n_rows, int64_t n_cols, int transposed,
                                     int64_t* counts, void* stream) {
  HREC_REQUIRE(n_rows >= 0 && n_cols >= 0 && row_begin >= 0, "synth_row_counts: negative size");
  HREC_REQUIRE(n_cols <= 0xffffffffll && row_begin + n_rows <= 0xffffffffll,
               "synth_row_counts: ids must be < 2^32");
  if (n_rows == 0) return HREC_OK;
  HREC_REQUIRE(counts != nullptr, "synth_row_counts: null counts");
  const int64_t blocks = (n_rows + 3) / 4;
  hipLaunchKernelGGL(synth_count_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), seed,
                     threshold, row_begin, n_rows, n_cols, transposed, counts);
  return check_launch("synth_count_kernel");
}

extern "C" int hrec_synth_fill(uint64_t seed, uint64_t seed2, uint64_t threshold, int64_t row_begin,
                               int64_t n_rows, int64_t n_cols, int transposed, int n_levels,
                               const int64_t* indptr, int32_t* indices, float* values, void* stream) {
  HREC_REQUIRE(n_rows >= 0 && n_cols >= 0 && row_begin >= 0, "synth_fill: negative size");
  HREC_REQUIRE(n_cols <= 0x7fffffffll && row_begin + n_rows <= 0xffffffffll,
               "synth_fill: column ids must fit int32");
  HREC_REQUIRE(n_levels > 0, "synth_fill: n_levels must be > 0");
  if (n_rows == 0) return HREC_OK;
  HREC_REQUIRE(indptr && indices && values, "synth_fill: null pointer");
  const int64_t blocks = (n_rows + 3) / 4;
  hipLaunchKernelGGL(synth_fill_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), seed,
                     seed2, threshold, row_begin, n_rows, n_cols, transposed, n_levels, indptr,
                     indices, values);
  return check_launch("synth_fill_kernel");
}

extern "C" size_t hrec_scan_workspace_bytes(int64_t n) { return scan_ws_bytes(n); }

extern "C" int hrec_exclusive_scan_i64(const int64_t* counts, int64_t n, int64_t* out, void* workspace,
                                       size_t workspace_bytes, void* stream) {
  HREC_REQUIRE(n >= 0, "exclusive_scan: n out of range");
  HREC_REQUIRE(out != nullptr, "exclusive_scan: null out");
  hipStream_t s = as_stream(stream);
  if (hipMemsetAsync(out, 0, sizeof(int64_t), s) != hipSuccess) return check_launch("scan memset");
  if (n == 0) return HREC_OK;
  HREC_REQUIRE(counts && workspace, "exclusive_scan: null pointer");
  const size_t need = hrec_scan_workspace_bytes(n);
  HREC_REQUIRE(workspace_bytes >= need, "exclusive_scan: workspace %zu < %zu", workspace_bytes, need);
  return scan_run<int64_t>(counts, out + 1, n, false, workspace, s);
}

extern "C" int hrec_als_init_factors(uint64_t seed, int64_t row_begin, int64_t n_rows, int k, int kp,
                                     float* out, void* stream) {
  HREC_REQUIRE(k >= 1 && k <= kp && hrec_factor_ld_ok(kp), "als_init_factors: bad k=%d kp=%d",
               k, kp);
  HREC_REQUIRE(n_rows >= 0 && row_begin >= 0, "als_init_factors: negative size");
  if (n_rows == 0) return HREC_OK;
  HREC_REQUIRE(out != nullptr, "als_init_factors: null out");
  const int64_t blocks = (n_rows + 3) / 4;
  hipLaunchKernelGGL(init_factors_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), seed,
                     row_begin, n_rows, k, kp, out);
  return check_launch("init_factors_kernel");
}
