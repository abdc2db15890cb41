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
#include <type_traits>

#include "common.h"

// Occupancy target of the half-sweep (waves per SIMD; caps VGPRs at 168 for
// 3) and the pipeline chunk (steps of 4 ratings) per accumulation mode.
#ifndef HREC_ALS_WAVES
#define HREC_ALS_WAVES 2
#endif
#ifndef HREC_ALS_CH0
#define HREC_ALS_CH0 8
#endif
#ifndef HREC_ALS_ABLATE
#define HREC_ALS_ABLATE 0  // timing-only builds: 1 = skip the solve, 2 = skip the MFMA Gramian
#endif
#ifndef HREC_ALS_BCAST_LDS
#define HREC_ALS_BCAST_LDS 1  // Cholesky column broadcast: 1 = LDS ds_read_b128, 0 = v_readlane
#endif
#ifndef HREC_ALS_FAST_RSQ
#define HREC_ALS_FAST_RSQ 1  // pivot 1/sqrt by v_rsq_f64 + one Newton step (else sqrt + divide)
#endif
#ifndef HREC_ALS_SOLVE
#define HREC_ALS_SOLVE 1  // 1 = blocked tile-layout Cholesky (MFMA trailing updates); 0 = row-per-lane
#endif
#ifndef HREC_ALS_SOLVE_UNROLL
#define HREC_ALS_SOLVE_UNROLL 8  // unroll of the two 64-step triangular-solve loops
#endif
#ifndef HREC_ALS_CH1
#define HREC_ALS_CH1 4
#endif
#ifndef HREC_ALS_PIPE
#define HREC_ALS_PIPE 1  // 1 = ring-prefetch gather with structured buffer loads; 0 = chunked flat loads
#endif
#ifndef HREC_ALS_PF
#define HREC_ALS_PF 8  // PIPE: gather prefetch distance in steps of 4 ratings
#endif

namespace hrec {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

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

// Structured buffer loads (buffer_load_dword* ... idxen offen): address =
// base + vindex * stride + voffset, with the hardware range check
// (vindex >= num_records reads as zero).
typedef int i4v __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ f4 sbuf_load_f4(i4v rsrc, int vindex, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.struct.buffer.load.v4f32");
__device__ f2 sbuf_load_f2(i4v rsrc, int vindex, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.struct.buffer.load.v2f32");
__device__ float sbuf_load_f1(i4v rsrc, int vindex, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.struct.buffer.load.f32");

template <int NT>
__device__ __forceinline__ Vec<NT> struct_load(i4v rsrc, int vindex, int voffset) {
  Vec<NT> v;
  if constexpr (NT == 4) {
    const f4 t = sbuf_load_f4(rsrc, vindex, voffset, 0, 0);
    v.x[0] = t.x, v.x[1] = t.y, v.x[2] = t.z, v.x[3] = t.w;
  } else if constexpr (NT == 2) {
    const f2 t = sbuf_load_f2(rsrc, vindex, voffset, 0, 0);
    v.x[0] = t.x, v.x[1] = t.y;
  } else {
    v.x[0] = sbuf_load_f1(rsrc, vindex, voffset, 0, 0);
  }
  return v;
}

#ifdef HREC_ALS_STAMPS
// Diagnostic build only: per-phase cycle sums (s_memtime) over all waves.
__device__ unsigned long long g_als_stamps[8];
#define STAMP(i)                                                                      \
  do {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                       \
    __builtin_amdgcn_sched_barrier(0);                                                \
    if (threadIdx.x == 0 && (i) > 0) atomicAdd(&g_als_stamps[(i) > 0 ? (i) - 1 : 0], _t - _stamp_prev); \
    _stamp_prev = _t;                                                                 \
  } while (0)
#define STAMP_DECL unsigned long long _stamp_prev = 0
#else
#define STAMP(i) \
  do {           \
  } while (0)
#define STAMP_DECL
#endif

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
__device__ __forceinline__ double solve_spd_rows_impl(double* __restrict__ A, double* __restrict__ col, double bi,
                                                      int lane) {
  STAMP_DECL;
  STAMP(0);
  const int i = lane < KP ? lane : KP - 1;
  double a[KP];
#pragma unroll
  for (int c = 0; c < KP; ++c) {
    const int hi = i > c ? i : c, lo = i > c ? c : i;
    a[c] = A[tri(hi) + lo];
  }
  STAMP(4);  // phase 4: row load from LDS
  double myrd = 0.0;  // lane j keeps 1 / L[j][j]
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    // pivot: lane j's diagonal is current (column j was updated first, via a
    // readlane, at step j-1 — the short critical path of the factorisation)
    const double piv = bcast(a[j], j);
#if HREC_ALS_FAST_RSQ
    double rs = __builtin_amdgcn_rsq(piv);
    rs = rs * fma(-0.5 * piv * rs, rs, 1.5);  // one Newton step: full f64 precision
    const double d = piv * rs;
#else
    const double d = sqrt(piv);
    const double rs = 1.0 / d;
#endif
    const double l = (lane == j) ? d : a[j] * rs;
    a[j] = l;
    myrd = (lane == j) ? rs : myrd;
    if (j + 1 < KP) a[j + 1] = fma(-l, bcast(l, j + 1), a[j + 1]);
#if HREC_ALS_BCAST_LDS
    // remaining columns: column j of L to LDS once, then wave-uniform
    // ds_read_b128 broadcasts (two entries per read), off the critical path.
    if (j + 2 < KP) {
      if (lane < KP) col[lane] = l;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int c0 = (j + 2) & ~1; c0 < KP; c0 += 2) {
        const double2 lc = *reinterpret_cast<const double2*>(col + c0);
        if (c0 > j + 1) a[c0] = fma(-l, lc.x, a[c0]);
        a[c0 + 1] = fma(-l, lc.y, a[c0 + 1]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
#else
#pragma unroll
    for (int c = j + 2; c < KP; ++c) a[c] = fma(-l, bcast(l, c), a[c]);
#endif
  }
  STAMP(5);  // phase 5: factorisation
  // forward: L y = b
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    const double yj = bcast(bi, j) * bcast(myrd, j);
    const double upd = fma(-a[j], yj, bi);
    bi = (lane == j) ? yj : ((lane > j) ? upd : bi);
  }
  STAMP(6);  // phase 6: forward substitution
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
  STAMP(7);  // phase 7: transpose + back substitution
  return bi;
}

// NT floats per lane (kp = 16*NT), CH steps of 4 nnz per pipeline chunk.
// MODE 0: v_mfma_f64_16x16x4_f64 accumulates the Gramian in f64 (Spark's
//         f64 NormalEquation, any row length).
// MODE 1: v_mfma_f32_16x16x4_f32 (2x the f64 matrix rate) accumulates each
//         chunk of 4*CH ratings in f32 (an exact f32 fma chain), and the chunk
//         partials are flushed into f64 accumulators — f64 summation across
//         chunks, f32 rounding only inside a chunk.
template <int NT, int CH, int MODE>
__global__ __launch_bounds__(64, HREC_ALS_WAVES) void als_half_sweep_f64_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ values, int64_t n_rows, const float* __restrict__ src, int64_t n_src,
    int k, double reg, float* __restrict__ dst) {
  constexpr int KP = 16 * NT;
  constexpr int NPAIR = NT * (NT + 1) / 2;
  constexpr int CHN = 4 * CH;  // nnz per chunk (<= 64)
#if HREC_ALS_SOLVE == 1
  __shared__ double Up[KP * (KP + 1) / 2];  // U, column-packed: U[tri(c) + q], q <= c
  __shared__ double stage[MODE == 1 ? 256 : 1];
  __shared__ __attribute__((aligned(16))) double colbuf[64];
  __shared__ double dsh[KP];  // pivots U[r][r]
  double* A = nullptr;
#else
  __shared__ double A[KP * (KP + 1) / 2];
  __shared__ __attribute__((aligned(16))) double colbuf[KP];
#endif
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

  STAMP_DECL;
  STAMP(0);
  d4 acc[NPAIR];
#pragma unroll
  for (int p = 0; p < NPAIR; ++p) acc[p] = d4{0.0, 0.0, 0.0, 0.0};
  f4 fa[NPAIR];
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

  // PIPE for kp = 64 (at kp <= 32 the scheduler hoists the unrolled window
  // into a spill; those sizes keep the chunked loop)
  if constexpr (HREC_ALS_PIPE && NT == 4) {
  // Ring pipeline over WINDOWS of 16 steps (64 nnz: one index and one rating
  // per lane). Step s's gather is issued PF steps ahead into ring slot
  // s % PF; the index reaches the lane group by ds_bpermute and feeds a
  // structured buffer load (vindex = source row, stride = one factor row,
  // voffset = this lane's 16-B column slice). Padding entries carry index -1:
  // the buffer range check returns zeros for them, so the loop has no
  // branches, masks or address arithmetic on the VALU.
  constexpr int PF = HREC_ALS_PF;
  static_assert(16 % PF == 0, "prefetch distance must divide the window");
  const int voff = NT * 4 * col;
  const int bp_addr = 4 * sub;  // ds_bpermute byte address of nnz (4s + sub) is 16 s + 4 sub
  const uint64_t sbase = (uint64_t)src;
  i4v rsrc;
  rsrc.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)sbase);
  rsrc.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(sbase >> 32) | ((KP * 4) << 16));
  rsrc.z = __builtin_amdgcn_readfirstlane((int)n_src);
  rsrc.w = 0x00020000;
  auto load_win = [&](int64_t w, int& ii, float& vv) {
    const int64_t p = beg + 64 * w + lane;
    const int64_t pc = p < end ? p : end - 1;
    const int iraw = indices[pc];
    const float vraw = values[pc];
    ii = p < end ? iraw : -1;
    vv = p < end ? vraw : 0.f;
  };
  auto bperm = [&](int win, int s) -> int { return __builtin_amdgcn_ds_bpermute(bp_addr + 16 * s, win); };
  const int64_t nsteps = (n + 3) >> 2;
  int iw0, iw1;
  float rw0, rw1;
  load_win(0, iw0, rw0);
  load_win(1, iw1, rw1);
  Vec<NT> ring[PF];
#pragma unroll
  for (int s = 0; s < PF; ++s) ring[s] = struct_load<NT>(rsrc, bperm(iw0, s), voff);
  int nidx = bperm(iw0, PF);  // source row of the next gather (one step ahead)
  for (int64_t w = 0;; ++w) {
    int iw2;
    float rw2;
    load_win(w + 2, iw2, rw2);
    bool stop = false;
    const int rem = __builtin_amdgcn_readfirstlane((int)(nsteps - 16 * w < 16 ? nsteps - 16 * w : 16));
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s >= rem) {  // wave-uniform (scalar) tail exit
        stop = true;
        break;
      }
      const Vec<NT> cur = ring[s % PF];
      double a[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) a[t] = (double)cur.x[t];
      ring[s % PF] = struct_load<NT>(rsrc, nidx, voff);
      nidx = (s + 1 + PF < 16) ? bperm(iw0, s + 1 + PF) : bperm(iw1, s + 1 + PF - 16);
      const float rf = __int_as_float(__builtin_amdgcn_ds_bpermute(bp_addr + 16 * s, __float_as_int(rw0)));
      const double rv = (double)rf;
      if (MODE == 1 && (s % HREC_ALS_CH1) == 0) {
#pragma unroll
        for (int p = 0; p < NPAIR; ++p) fa[p] = f4{0.f, 0.f, 0.f, 0.f};
      }
      int p = 0;
#pragma unroll
      for (int I = 0; I < NT; ++I) {
#pragma unroll
        for (int J = I; J < NT; ++J) {
          if (MODE == 0)
            acc[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[I], a[J], acc[p], 0, 0, 0);
          else
            fa[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.x[I], cur.x[J], fa[p], 0, 0, 0);
          ++p;
        }
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) bp[t] = fma(rv, a[t], bp[t]);
      if (MODE == 1 && ((s % HREC_ALS_CH1) == HREC_ALS_CH1 - 1 || s + 1 == rem)) {
#pragma unroll
        for (int p2 = 0; p2 < NPAIR; ++p2) {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) acc[p2][rr] += (double)fa[p2][rr];
        }
      }
    }
    if (stop || 16 * (w + 1) >= nsteps) break;
    iw0 = iw1;
    rw0 = rw1;
    iw1 = iw2;
    rw1 = rw2;
  }
  } else {
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
    if (MODE == 1) {
#pragma unroll
      for (int p = 0; p < NPAIR; ++p) fa[p] = f4{0.f, 0.f, 0.f, 0.f};
    }
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
          if (HREC_ALS_ABLATE == 2) {
            acc[p][0] += a[I] * a[J];  // ablation: no matrix cores
          } else if (MODE == 0)
            acc[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[I], a[J], acc[p], 0, 0, 0);
          else
            fa[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(buf[s].x[I], buf[s].x[J], fa[p], 0, 0, 0);
          ++p;
        }
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) bp[t] = fma(rv, a[t], bp[t]);
    }
    if (MODE == 1) {
#pragma unroll
      for (int p = 0; p < NPAIR; ++p) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) acc[p][rr] += (double)fa[p][rr];
      }
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
  }

  STAMP(1);  // phase 1: Gramian (gather + MFMA)
  // b: sum the four row-groups of lanes.
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    bp[t] += __shfl_xor(bp[t], 16, kWave);
    bp[t] += __shfl_xor(bp[t], 32, kWave);
  }
#if HREC_ALS_SOLVE == 1
  // ---- blocked Cholesky in the matrix-core tile layout -------------------
  // Work in the permuted basis q = 16*T + m  <->  physical column NT*m + T:
  // tile (I,J) of the accumulators is then block (I,J) of the permuted
  // Gramian (rows of block I, columns of block J, I <= J: the upper block
  // triangle). A symmetric permutation does not change the solution; b and
  // x are permuted on the way in and out. Factor A = U^T U block row by
  // block row: a 16-pivot panel step with one LANE PER COLUMN (compact,
  // fully in registers), then the trailing update of every later block
  // U_KM -= U_JK^T U_JM on the f64 matrix cores, straight from the
  // accumulator registers (the C/D layout of tile (J,K) is exactly the A/B
  // operand layout of the 4 k-steps). U accumulates, column-packed, in LDS
  // (U[tri(c) + q], q <= c) for the two triangular solves.
  (void)A;
  if (sub == 0) {
#pragma unroll
    for (int t = 0; t < NT; ++t) bsh[16 * t + col] = bp[t];  // permuted b
  }
  if (MODE == 1) {
    // f32 C/D map (row = 4*(lane>>4) + reg) -> f64 map (row = (lane>>4) + 4*reg)
#pragma unroll
    for (int p = 0; p < NPAIR; ++p) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) stage[(4 * sub + rr) * 16 + col] = acc[p][rr];
      __syncthreads();
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) acc[p][rr] = stage[(sub + 4 * rr) * 16 + col];
      __syncthreads();
    }
  }
  STAMP(2);  // phase 2: b + layout
  // lambda = numExplicits * regParam on the diagonal (1.0 on padding columns)
  const double lambda = (double)n * reg;
  {
    int p = 0;
#pragma unroll
    for (int I = 0; I < NT; ++I) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        if (sub + 4 * rr == col) acc[p][rr] += (NT * col + I < k) ? lambda : 1.0;
      }
      p += NT - I;
    }
  }
  // The factor is stored UNIT-DIAGONAL: Ut[r][c] = U[r][c] / U[r][r] (row
  // scaled), column-packed in LDS (Ut[tri(c) + r], r <= c), with the pivots
  // d_r = U[r][r] in dsh. Then U^T y = b, U x = y become
  //   Ut^T w = b,  v = D^-2 w,  Ut x = v        (w = D y)
  // and each of the 2 x KP substitution steps is one broadcast + one masked fma.
  double myrd = 0.0;  // lane c keeps 1 / U[c][c]
  auto pidx = [](int I, int K) { return I * NT - (I * (I - 1)) / 2 + (K - I); };
#pragma unroll
  for (int J = 0; J < NT; ++J) {
    // (a) block row J -> LDS (only q <= c: the upper triangle)
#pragma unroll
    for (int K = J; K < NT; ++K) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int q = 16 * J + sub + 4 * rr, c = 16 * K + col;
        if (q <= c) Up[tri(c) + q] = acc[pidx(J, K)][rr];
      }
    }
    __syncthreads();
    // (b) lane c >= 16J owns column c of block row J
    const int c = lane;
    const bool own = c >= 16 * J && c < KP;
    double a[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int q = 16 * J + m;
      a[m] = (own && q <= c) ? Up[tri(c) + q] : 0.0;
    }
    // (c) 16 pivots, right-looking, columns on lanes. The pivot row of U goes
    //     to LDS once per pivot and comes back as wave-uniform ds_read_b128
    //     pairs; row pv of Ut is written beside it.
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int pv = 16 * J + i;
      const double piv = bcast(a[i], pv);
      double rs = __builtin_amdgcn_rsq(piv);
      rs = rs * fma(-0.5 * piv * rs, rs, 1.5);  // one Newton step: full f64 precision
      const double d = piv * rs;
      a[i] = (c == pv) ? d : a[i] * rs;  // U[pv][c]
      myrd = (c == pv) ? rs : myrd;
      if (own && c > pv) Up[tri(c) + pv] = a[i] * rs;  // Ut[pv][c]
      if (c == pv) dsh[pv] = d;
      if (i < 15) {
        if (c < KP) colbuf[c] = a[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int m0 = (i + 1) & ~1; m0 < 16; m0 += 2) {
          const double2 u = *reinterpret_cast<const double2*>(colbuf + 16 * J + m0);
          if (m0 > i) a[m0] = fma(-u.x, a[i], a[m0]);
          a[m0 + 1] = fma(-u.y, a[i], a[m0 + 1]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
    }
    __syncthreads();
    // (e) U_JK = D_J Ut_JK (K > J) back into tile registers; (f) trailing
    //     update U_KM -= U_JK^T U_JM on the f64 matrix cores
    if (J + 1 < NT) {
      double dq[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) dq[rr] = dsh[16 * J + sub + 4 * rr];
#pragma unroll
      for (int K = J + 1; K < NT; ++K) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          acc[pidx(J, K)][rr] = Up[tri(16 * K + col) + 16 * J + sub + 4 * rr] * dq[rr];
      }
#pragma unroll
      for (int K = J + 1; K < NT; ++K) {
#pragma unroll
        for (int M = K; M < NT; ++M) {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            acc[pidx(K, M)] = __builtin_amdgcn_mfma_f64_16x16x4f64(-acc[pidx(J, K)][rr], acc[pidx(J, M)][rr],
                                                                    acc[pidx(K, M)], 0, 0, 0);
        }
      }
    }
  }
  STAMP(3);  // phase 3: factorisation
  // forward  Ut^T w = b   (step q: lanes c > q subtract Ut[q][c] * w_q)
  double bi = lane < KP ? bsh[lane] : 0.0;
#pragma unroll HREC_ALS_SOLVE_UNROLL
  for (int q = 0; q < KP; ++q) {
    const double u = Up[tri(lane < KP ? lane : KP - 1) + q];  // in bounds; used by lanes > q only
    const double wq = bcast(bi, q);
    if (lane > q) bi = fma(-u, wq, bi);
  }
  bi *= myrd * myrd;  // v = D^-2 w
  // back     Ut x = v     (step q: lanes c < q subtract Ut[c][q] * x_q)
#pragma unroll HREC_ALS_SOLVE_UNROLL
  for (int q = KP - 1; q >= 0; --q) {
    const double u = Up[tri(q) + (lane < KP ? lane : 0)];  // Ut[lane][q] for lane < q
    const double xq = bcast(bi, q);
    if (lane < q) bi = fma(-u, xq, bi);
  }
  STAMP(4);  // phase 4: triangular solves
  if (lane < KP) out[NT * (lane & 15) + (lane >> 4)] = (float)bi;
}
#else
  if (sub == 0) {
#pragma unroll
    for (int t = 0; t < NT; ++t) bsh[NT * col + t] = bp[t];
  }
  // Gramian -> packed lower triangle. C/D maps: f64 16x16x4 col = lane&15,
  // row = (lane>>4) + 4*reg; f32 16x16x4 col = lane&15, row = 4*(lane>>4) + reg.
  {
    int p = 0;
#pragma unroll
    for (int I = 0; I < NT; ++I) {
#pragma unroll
      for (int J = I; J < NT; ++J) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int pr = NT * (MODE == 0 ? sub + 4 * rr : 4 * sub + rr) + I;  // physical row
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

  STAMP(2);  // phase 2: b reduce + Gramian -> LDS
  // Spark CholeskySolver: ata[diag] += numExplicits * regParam.
  const double lambda = (double)n * reg;
  if (lane < KP) A[tri(lane) + lane] += (lane < k) ? lambda : 1.0;
  const double b_in = lane < KP ? bsh[lane] : 0.0;
  __syncthreads();
  const double x = HREC_ALS_ABLATE == 1 ? b_in + A[tri(lane < KP ? lane : 0)] : solve_spd_rows_impl<KP>(A, colbuf, b_in, lane);
  if (lane < KP) out[lane] = (float)x;
}
#endif

__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ in, int64_t rows,
                                                        int64_t cols, float* __restrict__ out, int64_t ld_out) {
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
    if (r < rows && c < cols) out[c * ld_out + r] = tile[tx][i];
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
  HREC_REQUIRE(accum_mode == 0 || accum_mode == 1, "als_half_sweep: accum_mode %d unsupported", accum_mode);
  HREC_REQUIRE(reg_param >= 0.0, "als_half_sweep: reg_param must be >= 0");
  if (n_rows == 0) return HREC_OK;
  HREC_REQUIRE(indptr && dst_factors, "als_half_sweep: null pointer");
  HREC_REQUIRE(n_src > 0 && src_factors && indices && values,
               "als_half_sweep: null source factors / CSR arrays");
  HREC_REQUIRE(n_src < 0x7fffffffll, "als_half_sweep: too many source rows for one launch");
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)n_rows), block(64);
#define HREC_SWEEP(NT, CH, M)                                                                      \
  hipLaunchKernelGGL((als_half_sweep_f64_kernel<NT, CH, M>), grid, block, 0, s, indptr, indices, values, \
                     n_rows, src_factors, n_src, k, reg_param, dst_factors)
  if (accum_mode == 0) {
    if (kp == 64) HREC_SWEEP(4, HREC_ALS_CH0, 0);
    else if (kp == 32) HREC_SWEEP(2, 8, 0);
    else HREC_SWEEP(1, 8, 0);
  } else {
    if (kp == 64) HREC_SWEEP(4, HREC_ALS_CH1, 1);
    else if (kp == 32) HREC_SWEEP(2, 4, 1);
    else HREC_SWEEP(1, 4, 1);
  }
#undef HREC_SWEEP
  return check_launch("als_half_sweep_f64_kernel");
}

extern "C" int hrec_transpose_f32(const float* in, int64_t rows, int64_t cols, float* out, int64_t ld_out,
                                  void* stream) {
  HREC_REQUIRE(rows >= 0 && cols >= 0, "transpose: negative size");
  HREC_REQUIRE(ld_out >= rows, "transpose: ld_out < rows");
  if (rows == 0 || cols == 0) return HREC_OK;
  HREC_REQUIRE(in && out, "transpose: null pointer");
  const dim3 grid((unsigned)((rows + 63) / 64), (unsigned)((cols + 63) / 64)), block(256);
  hipLaunchKernelGGL(transpose_kernel, grid, block, 0, as_stream(stream), in, rows, cols, out, ld_out);
  return check_launch("transpose_kernel");
}

#ifdef HREC_ALS_STAMPS
extern "C" int hrec_debug_als_stamps(unsigned long long* host_out, int reset) {
  if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_als_stamps), sizeof(g_als_stamps)) != hipSuccess) return -2;
  if (reset) {
    unsigned long long z[8] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_als_stamps), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 0;
}
#endif
