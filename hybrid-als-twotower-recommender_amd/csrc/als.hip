// K1: ALS half-sweep — CSR row gather -> f64 MFMA Gramian -> Cholesky solve.
//
// Replaces Spark 3.5.1 ALS.computeFactors / NormalEquation.add /
// CholeskySolver.solve [ext], reached from src/als_model.py:62 (als.fit).
// Per destination row r (one wave per row):
//   A = sum_j v_j v_j^T  (f64),  b = sum_j r_j v_j (f64),  n = #ratings
//   A[d][d] += reg * n, solve A x = b (Cholesky, f64), store f32.
//
// Gramian on the matrix cores: v_mfma_f64_16x16x4_f64 with the 4 nnz of a
// step as the K dimension. Each lane loads ONE 16-B vector (NT floats) of a
// gathered factor row: lane l holds row (l>>4) of the step, columns
// NT*(l&15) .. +NT-1. Column c = NT*m + T belongs to tile T at index m, so
// component T of the lane's vector is exactly the MFMA operand of tile T
// (A[i=l&15][k=l>>4], B[k=l>>4][j=l&15]) — no shuffles, fully coalesced
// 256-B row reads. Tile pair (I,J), I<=J, accumulates G[NT*m+I][NT*m'+J].
#include "common.h"

namespace hrec {

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NT>
struct Vec;
template <>
struct Vec<4> {
  float x[4];
  __device__ static Vec load(const float* p) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    return Vec{{t.x, t.y, t.z, t.w}};
  }
};
template <>
struct Vec<2> {
  float x[2];
  __device__ static Vec load(const float* p) {
    const float2 t = *reinterpret_cast<const float2*>(p);
    return Vec{{t.x, t.y}};
  }
};
template <>
struct Vec<1> {
  float x[1];
  __device__ static Vec load(const float* p) { return Vec{{*p}}; }
};

__device__ __forceinline__ int tri(int i) { return (i * (i + 1)) >> 1; }

// Wave-uniform broadcast of lane `src`'s double (two v_readlane_b32).
__device__ __forceinline__ double bcast(double v, int src) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)x, src);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// Solve (L L^T) x = b for the SPD matrix held as a packed lower triangle in
// LDS (row i at tri(i)), b_i in lane i. Right-looking Cholesky with the
// matrix in REGISTERS: lane i owns row i (a[c] = A[i][c]); every column
// broadcast is a v_readlane, so the O(k^3/6) update is pure VALU with static
// register indices (fully unrolled) and no LDS traffic. Entries right of the
// diagonal are never read, so lanes update them unmasked. The packed LDS
// array is reused once to transpose L for the back substitution.
template <int KP>
__device__ __forceinline__ double solve_spd_rows_impl(double* __restrict__ A, double bi, int lane) {
  const int i = lane < KP ? lane : KP - 1;
  double a[KP];
#pragma unroll
  for (int c = 0; c < KP; ++c) {
    const int hi = i > c ? i : c, lo = i > c ? c : i;
    a[c] = A[tri(hi) + lo];
  }
  double myrd = 0.0;  // lane j keeps 1 / L[j][j]
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    const double d = sqrt(bcast(a[j], j));
    const double rd = 1.0 / d;
    const double l = (lane == j) ? d : a[j] * rd;
    a[j] = l;
    myrd = (lane == j) ? rd : myrd;
#pragma unroll
    for (int c = j + 1; c < KP; ++c) a[c] = fma(-l, bcast(l, c), a[c]);
  }
  // forward: L y = b
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    const double yj = bcast(bi, j) * bcast(myrd, j);
    const double upd = fma(-a[j], yj, bi);
    bi = (lane == j) ? yj : ((lane > j) ? upd : bi);
  }
  // transpose L through LDS: lane i stores row i, then reads column i.
  __syncthreads();
  if (lane < KP) {
#pragma unroll
    for (int c = 0; c < KP; ++c)
      if (c <= lane) A[tri(lane) + c] = a[c];
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < KP; ++c) a[c] = (c >= i) ? A[tri(c) + i] : 0.0;  // a[c] = L[c][i]
  // backward: L^T x = y
#pragma unroll
  for (int j = KP - 1; j >= 0; --j) {
    const double xj = bcast(bi, j) * bcast(myrd, j);
    const double upd = fma(-a[j], xj, bi);
    bi = (lane == j) ? xj : ((lane < j) ? upd : bi);
  }
  return bi;
}

// NT floats per lane (kp = 16*NT), CH steps of 4 nnz per pipeline chunk.
template <int NT, int CH>
__global__ __launch_bounds__(64) void als_half_sweep_f64_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ values, int64_t n_rows, const float* __restrict__ src, int k,
    double reg, float* __restrict__ dst) {
  constexpr int KP = 16 * NT;
  constexpr int NPAIR = NT * (NT + 1) / 2;
  constexpr int CHN = 4 * CH;  // nnz per chunk (<= 64)
  __shared__ double A[KP * (KP + 1) / 2];
  __shared__ double bsh[KP];

  const int lane = threadIdx.x;
  const int sub = lane >> 4;  // which nnz of the step this lane loads
  const int col = lane & 15;  // which NT-column group
  const int64_t row = blockIdx.x;
  const int64_t beg = indptr[row];
  const int64_t end = indptr[row + 1];
  const int64_t n = end - beg;
  float* __restrict__ out = dst + row * KP;
  if (n == 0) {
    if (lane < KP) out[lane] = 0.f;
    return;
  }

  d4 acc[NPAIR];
#pragma unroll
  for (int p = 0; p < NPAIR; ++p) acc[p] = d4{0.0, 0.0, 0.0, 0.0};
  double bp[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) bp[t] = 0.0;

  // Chunk c's (index, rating) pairs live in lanes 0..CHN-1; padding entries
  // point at row 0 (always valid) with a zero mask so no load is predicated.
  auto load_iv = [&](int64_t base, int& ii, float& vv) {
    const int64_t p = base + (lane % CHN);
    const bool ok = (lane < CHN) && (p < end);
    ii = ok ? indices[p] : -1;
    vv = ok ? values[p] : 0.f;
  };
  auto gather = [&](Vec<NT> (&buf)[CH], int ii) {
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      const int idx = __shfl(ii, 4 * s + sub, kWave);
      const int safe = idx < 0 ? 0 : idx;
      Vec<NT> v = Vec<NT>::load(src + (int64_t)safe * KP + NT * col);
#pragma unroll
      for (int t = 0; t < NT; ++t) v.x[t] = idx < 0 ? 0.f : v.x[t];
      buf[s] = v;
    }
  };

  int i0, i1;
  float r0, r1;
  load_iv(beg, i0, r0);
  load_iv(beg + CHN, i1, r1);
  Vec<NT> buf[CH];
  gather(buf, i0);

  for (int64_t base = beg; base < end; base += CHN) {
    Vec<NT> nbuf[CH];
    const bool more = base + CHN < end;
    if (more) gather(nbuf, i1);
    int i2;
    float r2;
    load_iv(base + 2 * CHN, i2, r2);
#pragma unroll
    for (int s = 0; s < CH; ++s) {
      const double rv = (double)__shfl(r0, 4 * s + sub, kWave);
      double a[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) a[t] = (double)buf[s].x[t];
      int p = 0;
#pragma unroll
      for (int I = 0; I < NT; ++I) {
#pragma unroll
        for (int J = I; J < NT; ++J) {
          acc[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[I], a[J], acc[p], 0, 0, 0);
          ++p;
        }
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) bp[t] = fma(rv, a[t], bp[t]);
    }
    if (more) {
#pragma unroll
      for (int s = 0; s < CH; ++s) buf[s] = nbuf[s];
    }
    i0 = i1;
    r0 = r1;
    i1 = i2;
    r1 = r2;
  }

  // b: sum the four row-groups of lanes.
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    bp[t] += __shfl_xor(bp[t], 16, kWave);
    bp[t] += __shfl_xor(bp[t], 32, kWave);
  }
  if (sub == 0) {
#pragma unroll
    for (int t = 0; t < NT; ++t) bsh[NT * col + t] = bp[t];
  }
  // Gramian -> packed lower triangle. f64 16x16x4 C/D map:
  // col = lane&15, row = (lane>>4) + 4*reg.
  {
    int p = 0;
#pragma unroll
    for (int I = 0; I < NT; ++I) {
#pragma unroll
      for (int J = I; J < NT; ++J) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int pr = NT * (sub + 4 * rr) + I;  // physical row
          const int qc = NT * col + J;             // physical column
          const double v = acc[p][rr];
          if (I != J || pr >= qc) {
            const int hi = pr > qc ? pr : qc;
            const int lo = pr > qc ? qc : pr;
            A[tri(hi) + lo] = v;
          }
        }
        ++p;
      }
    }
  }
  __syncthreads();

  // Spark CholeskySolver: ata[diag] += numExplicits * regParam.
  const double lambda = (double)n * reg;
  if (lane < KP) A[tri(lane) + lane] += (lane < k) ? lambda : 1.0;
  const double b_in = lane < KP ? bsh[lane] : 0.0;
  __syncthreads();
  const double x = solve_spd_rows_impl<KP>(A, b_in, lane);
  if (lane < KP) out[lane] = (float)x;
}

__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ in, int64_t rows,
                                                        int64_t cols, float* __restrict__ out) {
  __shared__ float tile[64][65];
  const int64_t r0 = (int64_t)blockIdx.x * 64;
  const int64_t c0 = (int64_t)blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < rows && c < cols) ? in[r * cols + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, r = r0 + tx;
    if (r < rows && c < cols) out[c * rows + r] = tile[tx][i];
  }
}

}  // namespace hrec

using namespace hrec;

extern "C" int hrec_als_half_sweep(const int64_t* indptr, const int32_t* indices, const float* values,
                                   int64_t n_rows, const float* src_factors, int64_t n_src, int k,
                                   int kp, double reg_param, int accum_mode, float* dst_factors,
                                   void* stream) {
  HREC_REQUIRE(kp == 16 || kp == 32 || kp == 64, "als_half_sweep: kp must be 16, 32 or 64 (got %d)", kp);
  HREC_REQUIRE(k >= 1 && k <= kp, "als_half_sweep: need 1 <= k <= kp (k=%d kp=%d)", k, kp);
  HREC_REQUIRE(n_rows >= 0 && n_src >= 0, "als_half_sweep: negative size");
  HREC_REQUIRE(n_rows < 0x7fffffffll, "als_half_sweep: too many rows for one launch");
  HREC_REQUIRE(accum_mode == 0, "als_half_sweep: accum_mode %d unsupported", accum_mode);
  HREC_REQUIRE(reg_param >= 0.0, "als_half_sweep: reg_param must be >= 0");
  if (n_rows == 0) return HREC_OK;
  HREC_REQUIRE(indptr && dst_factors, "als_half_sweep: null pointer");
  HREC_REQUIRE(n_src > 0 && src_factors && indices && values,
               "als_half_sweep: null source factors / CSR arrays");
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)n_rows), block(64);
  switch (kp) {
    case 64:
      hipLaunchKernelGGL((als_half_sweep_f64_kernel<4, 8>), grid, block, 0, s, indptr, indices, values,
                         n_rows, src_factors, k, reg_param, dst_factors);
      break;
    case 32:
      hipLaunchKernelGGL((als_half_sweep_f64_kernel<2, 8>), grid, block, 0, s, indptr, indices, values,
                         n_rows, src_factors, k, reg_param, dst_factors);
      break;
    default:
      hipLaunchKernelGGL((als_half_sweep_f64_kernel<1, 8>), grid, block, 0, s, indptr, indices, values,
                         n_rows, src_factors, k, reg_param, dst_factors);
      break;
  }
  return check_launch("als_half_sweep_f64_kernel");
}

extern "C" int hrec_transpose_f32(const float* in, int64_t rows, int64_t cols, float* out, void* stream) {
  HREC_REQUIRE(rows >= 0 && cols >= 0, "transpose: negative size");
  if (rows == 0 || cols == 0) return HREC_OK;
  HREC_REQUIRE(in && out, "transpose: null pointer");
  const dim3 grid((unsigned)((rows + 63) / 64), (unsigned)((cols + 63) / 64)), block(256);
  hipLaunchKernelGGL(transpose_kernel, grid, block, 0, as_stream(stream), in, rows, cols, out);
  return check_launch("transpose_kernel");
}
