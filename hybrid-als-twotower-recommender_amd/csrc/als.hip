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
#define HREC_ALS_ABLATE 0  // timing-only builds: 1 = skip factor+solve, 3 = skip the back substitution, 4 = skip the Gramian
#endif
#ifndef HREC_ALS_SOLVE_UNROLL
#define HREC_ALS_SOLVE_UNROLL 8  // unroll of the two 64-step triangular-solve loops
#endif
#ifndef HREC_ALS_CH1
#define HREC_ALS_CH1 4
#endif
#ifndef HREC_ALS_INTCVT
#define HREC_ALS_INTCVT 0  // 1 = Gramian operands f32 -> f64 by 32-bit integer ops (measured slower)
#endif
#ifndef HREC_ALS_RLPANEL
#define HREC_ALS_RLPANEL 0  // 1 = pivot-row entries by v_readlane, 2 = only the next pivot's (both measured slower)
#endif
#ifndef HREC_ALS_DIAG4
// diagonal Gramian tiles as 3 x v_mfma_f64_4x4x4_4b (3/4 of the 16x16x4 work):
// 3 = rotated operands gathered from memory (default); 1 / 2 = rotated by DPP /
// ds_bpermute (measured slower); 0 = whole 16x16x4 diagonal tiles
#define HREC_ALS_DIAG4 3
#endif
#ifndef HREC_ALS_PIPE
#define HREC_ALS_PIPE 1  // 1 = ring-prefetch gather with structured buffer loads; 0 = chunked flat loads
#endif
#ifndef HREC_ALS_PF
#define HREC_ALS_PF 8  // PIPE: gather prefetch distance in steps of 4 ratings
#endif
#ifndef HREC_ALS_PF64
#define HREC_ALS_PF64 4  // prefetch distance of f64-source gathers (steps)
#endif
#ifndef HREC_ALS_PAIR8
#define HREC_ALS_PAIR8 2  // DIAG4 = 3: two diagonal tiles share one rotation-by-8 product (2: pairs (0,2), (1,3) by half-width loads)
#endif
#ifndef HREC_ALS_ROT1DPP
#define HREC_ALS_ROT1DPP 1  // f32 sources: rotation by 4 by DPP moves of the converted operands (0: rotated load + conversion)
#endif
#ifndef HREC_ALS_ROT1DPP64
#define HREC_ALS_ROT1DPP64 0  // f64 sources: rotation by 4 by DPP moves of the gathered operands (0: rotated loads; 1 measured 41.6 -> 41.9 ms user side, bit-identical)
#endif
#ifndef HREC_ALS_PR
#define HREC_ALS_PR 2  // DIAG4 = 3: prefetch distance of the rotated loads (steps)
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

// Four f64 source-factor columns (32 B) of one gathered row: two 16-B
// structured loads (S64 gathers: source factors kept in f64, no conversion).
struct VecD {
  double x[4];
};
__device__ __forceinline__ VecD struct_load_d(i4v rsrc, int vindex, int voffset) {
  const f4 lo = sbuf_load_f4(rsrc, vindex, voffset, 0, 0);
  const f4 hi = sbuf_load_f4(rsrc, vindex, voffset + 16, 0, 0);
  VecD v;
  v.x[0] = __hiloint2double(__float_as_int(lo.y), __float_as_int(lo.x));
  v.x[1] = __hiloint2double(__float_as_int(lo.w), __float_as_int(lo.z));
  v.x[2] = __hiloint2double(__float_as_int(hi.y), __float_as_int(hi.x));
  v.x[3] = __hiloint2double(__float_as_int(hi.w), __float_as_int(hi.z));
  return v;
}

// Two f64 source-factor columns (16 B).
struct VecD2 {
  double x[2];
};
__device__ __forceinline__ VecD2 struct_load_d2(i4v rsrc, int vindex, int voffset) {
  const f4 t = sbuf_load_f4(rsrc, vindex, voffset, 0, 0);
  VecD2 v;
  v.x[0] = __hiloint2double(__float_as_int(t.y), __float_as_int(t.x));
  v.x[1] = __hiloint2double(__float_as_int(t.w), __float_as_int(t.z));
  return v;
}

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
// Diagnostic builds only: per-phase cycle sums (s_memtime) over all waves.
__device__ unsigned long long g_als_stamps[8];
#endif
#ifdef HREC_ALS_STAMPS
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

// f32 -> f64 from the bit fields with 32-bit integer ops only: v_cvt_f64_f32
// runs on the f64 pipe, which the Gramian's f64 MFMAs keep busy (f64 VALU ops
// do not co-execute with them; integer ops do). Exact for normal numbers and
// zeros; f32 subnormals (|x| < 2^-126) become zero; inf/NaN are not factor
// values (Spark's factors are finite).
__device__ __forceinline__ double f32_to_f64_int(float x) {
  const uint32_t u = __float_as_uint(x);
  const uint32_t em = u & 0x7fffffffu;
  const bool normal = (u & 0x7f800000u) != 0u;
  const uint32_t hi = (u & 0x80000000u) | (normal ? (em >> 3) + 0x38000000u : 0u);
  const uint32_t lo = normal ? em << 29 : 0u;
  return __hiloint2double((int)hi, (int)lo);
}

__device__ __forceinline__ double gram_cvt(float x) {
  if constexpr (HREC_ALS_INTCVT) return f32_to_f64_int(x);
  return (double)x;
}

// x of lane (l & 48) | ((l + 16 - N) & 15): a rotation inside each 16-lane
// row (DPP row_ror:N on both halves of the double).
template <int N>
__device__ __forceinline__ double row_ror(double x) {
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_mov_dpp((int)v, 0x120 + N, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(v >> 32), 0x120 + N, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// c ? x : y on a double as two 32-bit selects (v_cndmask_b32).
__device__ __forceinline__ double sel64(bool c, double x, double y) {
  const long long a = __double_as_longlong(x), b = __double_as_longlong(y);
  const int lo = c ? (int)a : (int)b, hi = c ? (int)(a >> 32) : (int)(b >> 32);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// Wave-uniform broadcast of lane `src`'s double (two v_readlane_b32).
__device__ __forceinline__ double bcast(double v, int src) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)x, src);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// Orders this wave's LDS accesses around a point (one wave owns each LDS
// slice; a wave's LDS operations complete in issue order).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Per-wave LDS slice of the half-sweep (doubles).
template <int KP>
struct RowLds {
  static constexpr int kUp = KP * (KP + 1) / 2;  // Ut, column-packed
  // Up doubles as the MODE 1 re-layout stage (256); keep colbuf 16-B aligned
  static constexpr int kUpPad = ((kUp > 256 ? kUp : 256) + 1) & ~1;
  static constexpr int kSize = kUpPad + 128 + 3 * KP;
};

// Gramian + rhs of one destination row on one wave (lane = 0..63):
// acc = sum_j v_j v_j^T (tile layout, + n*reg on the diagonal), b -> bsh.
// NT floats per lane (kp = 16*NT), CH steps of 4 nnz per pipeline chunk.
// MODE 0: v_mfma_f64_16x16x4_f64 accumulates the Gramian in f64 (Spark's
//         f64 NormalEquation, any row length).
// MODE 1: v_mfma_f32_16x16x4_f32 (2x the f64 matrix rate) accumulates each
//         chunk of 16 ratings in f32 (an exact f32 fma chain), and the chunk
//         partials are flushed into f64 accumulators — f64 summation across
//         chunks, f32 rounding only inside a chunk.
struct NoHook {
  __device__ void operator()() const {}
};

// `before_lds` runs once the row's Gramian is in registers, before the first
// LDS write (b, MODE 1 re-layout) — a no-op in the product kernel (the
// producer/consumer splits that waited there measured slower).
template <int NT, int CH, int MODE, typename Hook = NoHook, bool S64 = false>
__device__ __forceinline__ void gram_row(int64_t beg, int64_t end, int lane, const int32_t* __restrict__ indices,
                                         const float* __restrict__ values, const float* __restrict__ src,
                                         int64_t n_src, int k, double reg, d4 (&acc)[NT * (NT + 1) / 2],
                                         double* __restrict__ bsh, double* __restrict__ stage,
                                         Hook before_lds = Hook()) {
  constexpr int KP = 16 * NT;
  constexpr int NPAIR = NT * (NT + 1) / 2;
  constexpr int CHN = 4 * CH;  // nnz per chunk (<= 64)
  const int sub = lane >> 4;  // which nnz of the step this lane loads
  const int col = lane & 15;  // which NT-column group
  const int64_t n = end - beg;

  STAMP_DECL;
  STAMP(0);
#pragma unroll
  for (int p = 0; p < NPAIR; ++p) acc[p] = d4{0.0, 0.0, 0.0, 0.0};
  if constexpr (HREC_ALS_ABLATE == 4) {  // timing-only: factor/solve without the Gramian (SPD stand-in)
#pragma unroll
    for (int I = 0, p = 0; I < NT; p += NT - I, ++I)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) acc[p][rr] = (sub + 4 * rr == col) ? 1.0 + reg * (double)n : 0.0;
    if (lane < KP) bsh[lane] = 1.0;
    wave_lds_sync();
    return;
  }
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
  constexpr int PF = S64 ? HREC_ALS_PF64 : HREC_ALS_PF;  // f64 sources sit in the MALL: shorter distance
  static_assert(16 % PF == 0, "prefetch distance must divide the window");
  static_assert(!S64 || (NT == 4 && MODE == 0 && (HREC_ALS_DIAG4 == 0 || HREC_ALS_DIAG4 == 3)),
                "f64 sources: kp 64, f64 accumulation only");
  const int voff = (S64 ? 8 : 4) * NT * col;
  const int bp_addr = 4 * sub;  // ds_bpermute byte address of nnz (4s + sub) is 16 s + 4 sub
  const uint64_t sbase = (uint64_t)src;
  i4v rsrc;
  rsrc.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)sbase);
  rsrc.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(sbase >> 32) | ((KP * (S64 ? 8 : 4)) << 16));
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
  using RingT = std::conditional_t<S64, VecD, Vec<NT>>;
  auto ring_load = [&](int vi) -> RingT {
    if constexpr (S64) return struct_load_d(rsrc, vi, voff);
    else return struct_load<NT>(rsrc, vi, voff);
  };
  RingT ring[PF];
#pragma unroll
  for (int s = 0; s < PF; ++s) ring[s] = ring_load(bperm(iw0, s));
  int nidx = bperm(iw0, PF);  // source row of the next gather (one step ahead)
  // DIAG4: a diagonal tile's 16 x 16 block is 16 sub-blocks of 4 x 4, of
  // which 10 are distinct (symmetry). v_mfma_f64_4x4x4_4b runs 4 independent
  // 4 x 4 x 4 blocks at the 16x16x4 rate (16 vs 64 cycles, measured:
  // scripts/micro/mfma_f64_rate.hip); with A = B = the lane's operand it
  // yields the 4 diagonal sub-blocks (b, b), with B rotated by 4 / 8 lanes
  // inside each 16-lane row the sub-blocks (b, b + 1) and (b, b + 2) mod 4:
  // all 10, in 3/4 of the 16x16x4 time.
  // DIAG4 = 1 rotates with DPP moves at the step itself; DIAG4 = 2 converts
  // the next step's operands one step ahead and rotates them by ds_bpermute
  // (LDS path), so the rotations have a whole step to land.
  // DIAG4 = 3 gathers the rotated operands from memory instead: two more
  // 16-B structured loads per step (the same source rows, the column slices
  // of lane col + 4 and col + 8), PR steps ahead — no cross-lane moves.
  constexpr bool kDiag4 = HREC_ALS_DIAG4 && MODE == 0;
  constexpr bool kAhead = HREC_ALS_DIAG4 == 2 && MODE == 0;
  constexpr bool kMemRot = HREC_ALS_DIAG4 == 3 && MODE == 0;
  constexpr int PR = kMemRot ? HREC_ALS_PR : 1;  // rotated-load prefetch distance (steps)
  constexpr bool kRot1Dpp = kMemRot && (S64 ? HREC_ALS_ROT1DPP64 : HREC_ALS_ROT1DPP);
  static_assert(PR < PF, "rotated loads are issued from the current windows");
  const int voff1 = (S64 ? 8 : 4) * NT * ((col + 4) & 15), voff2 = (S64 ? 8 : 4) * NT * ((col + 8) & 15);
  auto rot_load = [&](int vi, int vo) -> RingT {
    if constexpr (S64) return struct_load_d(rsrc, vi, vo);
    else return struct_load<NT>(rsrc, vi, vo);
  };
  // PAIR8 = 2: the shared rotation-by-8 product pairs tiles (0, 2) and
  // (1, 3), whose operands are adjacent components: lanes col < 8 need
  // components {0, 1}, lanes col >= 8 {2, 3} — of the own slice (A) and of
  // the col + 8 slice (B). Two half-width loads at a per-lane offset deliver
  // exactly those, so no lane selects are needed.
  constexpr bool kPairL = kMemRot && HREC_ALS_PAIR8 == 2 && NT == 4;
  using PairT = std::conditional_t<S64, VecD2, Vec<2>>;
  const int hoff = (lane & 8) ? (S64 ? 16 : 8) : 0;
  auto pair_load = [&](int vi, int vo) -> PairT {
    if constexpr (S64) return struct_load_d2(rsrc, vi, vo);
    else return struct_load<2>(rsrc, vi, vo);
  };
  RingT rot1[PR], rot2[PR];
  PairT rotA[PR], rotB[PR];
  if constexpr (kMemRot) {
#pragma unroll
    for (int q = 0; q < PR; ++q) {
      const int vi = bperm(iw0, q);
      if constexpr (!kRot1Dpp) rot1[q] = rot_load(vi, voff1);
      if constexpr (kPairL) {
        rotA[q] = pair_load(vi, voff + hoff);
        rotB[q] = pair_load(vi, voff2 + hoff);
      } else {
        rot2[q] = rot_load(vi, voff2);
      }
    }
  }
  double dg[NT][3];
#pragma unroll
  for (int t = 0; t < NT; ++t) dg[t][0] = dg[t][1] = dg[t][2] = 0.0;
  // PAIR8 (DIAG4 = 3): the rotation-by-8 product of a diagonal tile has 2
  // distinct sub-blocks in its 4 blocks, so tiles 2P and 2P + 1 share one
  // v_mfma_f64_4x4x4_4b: blocks 0, 1 (lanes with col < 8) take tile 2P's
  // operands, blocks 2, 3 tile 2P + 1's (one conversion instead of two)
  constexpr bool kPair8 = kMemRot && HREC_ALS_PAIR8 && NT % 2 == 0;
  const bool hi8 = (lane & 8) != 0;
  double dc[NT / 2 > 0 ? NT / 2 : 1];
#pragma unroll
  for (int t = 0; t < (NT / 2 > 0 ? NT / 2 : 1); ++t) dc[t] = 0.0;
  const int ra1 = 4 * ((lane & 48) | ((lane + 4) & 15)), ra2 = 4 * ((lane & 48) | ((lane + 8) & 15));
  auto bperm64 = [](double x, int addr) {
    const long long v = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_ds_bpermute(addr, (int)v);
    const int hi = __builtin_amdgcn_ds_bpermute(addr, (int)(v >> 32));
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
  };
  double an[NT], r1n[NT], r2n[NT];  // kAhead: the next step's operands
  if constexpr (kAhead) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      an[t] = gram_cvt(ring[0].x[t]);
      r1n[t] = bperm64(an[t], ra1);
      r2n[t] = bperm64(an[t], ra2);
    }
  }
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
      const RingT cur = ring[s % PF];
      double a[NT], ar1[NT], ar2[NT], apair[NT / 2 > 0 ? NT / 2 : 1];
      if constexpr (kAhead) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          a[t] = an[t];
          ar1[t] = r1n[t];
          ar2[t] = r2n[t];
        }
      } else {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          if constexpr (S64) a[t] = cur.x[t];
          else a[t] = gram_cvt(cur.x[t]);
        }
      }
      ring[s % PF] = ring_load(nidx);
      if constexpr (kMemRot) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          if constexpr (S64) {
            ar1[t] = kRot1Dpp ? row_ror<12>(a[t]) : rot1[s % PR].x[t];
            if constexpr (!kPair8) ar2[t] = rot2[s % PR].x[t];
          } else {
            // ROT1DPP: the rotation by 4 lanes of the converted operand (two
            // 32-bit DPP moves) instead of a converted rotated load
            ar1[t] = kRot1Dpp ? row_ror<12>(a[t]) : gram_cvt(rot1[s % PR].x[t]);
            if constexpr (!kPair8) ar2[t] = gram_cvt(rot2[s % PR].x[t]);
          }
        }
        if constexpr (kPairL) {
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            if constexpr (S64) {
              apair[t] = rotA[s % PR].x[t];
              ar2[t] = rotB[s % PR].x[t];
            } else {
              apair[t] = gram_cvt(rotA[s % PR].x[t]);
              ar2[t] = gram_cvt(rotB[s % PR].x[t]);
            }
          }
        } else if constexpr (kPair8) {
#pragma unroll
          for (int t = 0; t < NT / 2; ++t) {
            if constexpr (S64) ar2[t] = sel64(hi8, rot2[s % PR].x[2 * t + 1], rot2[s % PR].x[2 * t]);
            else ar2[t] = gram_cvt(hi8 ? rot2[s % PR].x[2 * t + 1] : rot2[s % PR].x[2 * t]);
            apair[t] = sel64(hi8, a[2 * t + 1], a[2 * t]);
          }
        }
        const int vr = (s + PR < 16) ? bperm(iw0, s + PR) : bperm(iw1, s + PR - 16);
        if constexpr (!kRot1Dpp) rot1[s % PR] = rot_load(vr, voff1);
        if constexpr (kPairL) {
          rotA[s % PR] = pair_load(vr, voff + hoff);
          rotB[s % PR] = pair_load(vr, voff2 + hoff);
        } else {
          rot2[s % PR] = rot_load(vr, voff2);
        }
      }
      if constexpr (kAhead) {
        const Vec<NT> nx = ring[(s + 1) % PF];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          an[t] = gram_cvt(nx.x[t]);
          r1n[t] = bperm64(an[t], ra1);
          r2n[t] = bperm64(an[t], ra2);
        }
      }
      nidx = (s + 1 + PF < 16) ? bperm(iw0, s + 1 + PF) : bperm(iw1, s + 1 + PF - 16);
      const float rf = __int_as_float(__builtin_amdgcn_ds_bpermute(bp_addr + 16 * s, __float_as_int(rw0)));
      const double rv = gram_cvt(rf);
      if (MODE == 1 && (s % HREC_ALS_CH1) == 0) {
#pragma unroll
        for (int p = 0; p < NPAIR; ++p) fa[p] = f4{0.f, 0.f, 0.f, 0.f};
      }
      int p = 0;
#pragma unroll
      for (int I = 0; I < NT; ++I) {
#pragma unroll
        for (int J = I; J < NT; ++J) {
          if (MODE == 0) {
            if (kDiag4 && I == J) {
              dg[I][0] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[I], a[I], dg[I][0], 0, 0, 0);
              dg[I][1] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[I], (kAhead || kMemRot) ? ar1[I] : row_ror<12>(a[I]),
                                                            dg[I][1], 0, 0, 0);
              if constexpr (kPairL) {  // tiles I and I + 2
                if (I < 2) dc[I] = __builtin_amdgcn_mfma_f64_4x4x4f64(apair[I], ar2[I], dc[I], 0, 0, 0);
              } else if constexpr (kPair8) {
                if (I % 2 == 0)
                  dc[I / 2] = __builtin_amdgcn_mfma_f64_4x4x4f64(apair[I / 2], ar2[I / 2], dc[I / 2], 0, 0, 0);
              } else {
                dg[I][2] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[I], (kAhead || kMemRot) ? ar2[I] : row_ror<8>(a[I]),
                                                              dg[I][2], 0, 0, 0);
              }
            } else {
              acc[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[I], a[J], acc[p], 0, 0, 0);
            }
          } else {
            fa[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.x[I], cur.x[J], fa[p], 0, 0, 0);
          }
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
  if constexpr (kDiag4) {
    // 4x4x4 block C[i][j] of block q sits at lane 16 i + 4 q + j and holds
    // G[4q + i][4((q + s) & 3) + j] for rotation s; write it and its mirror
    // into a 16 x 16 LDS image, read back the 16x16x4 C layout (one pass per
    // diagonal tile and row)
    const int i4 = lane >> 4, q4 = (lane >> 2) & 3, j4 = lane & 3;
#pragma unroll
    for (int I = 0, p = 0; I < NT; p += NT - I, ++I) {
#pragma unroll
      for (int sh = 0; sh < 3; ++sh) {
        const int r = 4 * q4 + i4, c = 4 * ((q4 + sh) & 3) + j4;
        if (kPair8 && sh == 2) {  // this tile's blocks of the shared product (with their mirrors: all 4)
          // the other tile's lanes write the same values to the junk slots 256, 257
          const bool mine = kPairL ? (q4 >= 2) == (I >= 2) : (q4 >= 2) == (I % 2 == 1);
          const double v = kPairL ? dc[I & 1] : dc[I / 2];
          stage[mine ? r * 16 + c : 256] = v;
          stage[mine ? c * 16 + r : 257] = v;
          continue;
        }
        stage[r * 16 + c] = dg[I][sh];
        stage[c * 16 + r] = dg[I][sh];
      }
      wave_lds_sync();
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) acc[p][rr] = stage[(sub + 4 * rr) * 16 + col];
      wave_lds_sync();
    }
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
          if (MODE == 0)
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
  // operand layout of the 4 k-steps).
  before_lds();
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
      wave_lds_sync();
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) acc[p][rr] = stage[(sub + 4 * rr) * 16 + col];
      wave_lds_sync();
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
}

// Factor + solve of one row's normal equations on one wave: acc (tile layout,
// consumed), b in bsh; Ut in Up (KP(KP+1)/2), row buffers and pivots in
// scratch (128 + 2 KP); x -> out[0..KP).
template <int NT>
__device__ __forceinline__ void factor_row(int lane, d4 (&acc)[NT * (NT + 1) / 2], double* __restrict__ Up,
                                           double* __restrict__ scratch, const double* __restrict__ bsh,
                                           float* __restrict__ out) {
  constexpr int KP = 16 * NT;
  constexpr int NPAIR = NT * (NT + 1) / 2;
  double* __restrict__ colbuf = scratch;    // two 64-entry row buffers (16-B aligned)
  double* __restrict__ dsh = colbuf + 128;  // pivots d_r
  double* __restrict__ rdsh = dsh + KP;     // 1 / d_r
  const int sub = lane >> 4, col = lane & 15;
  STAMP_DECL;
  STAMP(0);
  if constexpr (HREC_ALS_ABLATE == 1) {  // timing-only: Gramian without factor/solve
    double sum = 0.0;
#pragma unroll
    for (int p = 0; p < NPAIR; ++p) sum += acc[p][0] + acc[p][1] + acc[p][2] + acc[p][3];
    wave_lds_sync();
    if (lane < KP) out[lane] = (float)(sum + bsh[lane]);
    return;
  }
  // A = Ut^T D Ut with Ut unit upper triangular, stored column-packed in LDS
  // (Ut[tri(c) + r], r <= c), pivots d_r in dsh and 1/d_r in rdsh. A x = b is
  //   Ut^T w = b,  v = D^-1 w,  Ut x = v
  // and each of the 2 x KP substitution steps is one broadcast + one masked fma.
  // (Spark's dppsv factors A = U^T U with U = D^1/2 Ut: the same solution.)
  auto pidx = [](int I, int K) { return I * NT - (I * (I - 1)) / 2 + (K - I); };
  // The forward substitution Ut^T w = b rides along the panels: at pivot pv
  // lane c > pv holds Ut[pv][c] (= ut) and w_pv is lane pv's b, final since
  // pivot pv - 1, so b_c -= Ut[pv][c] w_pv is one broadcast + one fma off the
  // panel's critical chain — the same operands in the same (pv ascending)
  // order as a separate substitution loop, so the same bits.
  double bs = 0.0;
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
    wave_lds_sync();
    if (J == 0) bs = lane < KP ? bsh[lane] : 0.0;
    // (b) lane c >= 16J owns column c of block row J
    const int c = lane;
    const bool own = c >= 16 * J && c < KP;
    double a[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int q = 16 * J + m;
      if constexpr (HREC_ALS_RLPANEL) {
        // the diagonal block's lanes also hold its lower triangle (A[c][q] by
        // symmetry), so column pv carries the pivot row of the block
        a[m] = !own ? 0.0 : q <= c ? Up[tri(c) + q] : c < 16 * J + 16 ? Up[tri(q) + c] : 0.0;
      } else {
        a[m] = (own && q <= c) ? Up[tri(c) + q] : 0.0;
      }
    }
    // (c) 16 pivots of A = Ut^T D Ut (LDL^T: no square roots), right-looking,
    //     columns on lanes. The unscaled pivot row goes to LDS (alternating
    //     buffers) and comes back as wave-uniform ds_read_b128 pairs; the next
    //     pivot is formed on its own lane ahead of that round trip (its update
    //     needs only the lane's own entries), so the per-pivot critical path is
    //     rcp -> Newton -> scale -> fma -> readlane.
    double piv = bcast(a[0], 16 * J);
    if constexpr (HREC_ALS_RLPANEL) {
      // Pivot pv's row within the block, A[pv][16J + m] (m > i), is lane pv's
      // own column entries A[16J + m][pv] (the Schur complement stays
      // symmetric): read by v_readlane at the start of the pivot, so the
      // per-pivot critical path is rcp -> Newton -> scale -> fma -> readlane,
      // with no LDS store/load round trip.
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int pv = 16 * J + i;
        double u[16];
#pragma unroll
        for (int m0 = i + 1; m0 < 16; ++m0) u[m0] = bcast(a[m0], pv);
        const double r0 = __builtin_amdgcn_rcp(piv);
        const double r = fma(r0, fma(-piv, r0, 1.0), r0);
        const double ut = a[i] * r;  // Ut[pv][c]
        if (own && c > pv) Up[tri(c) + pv] = ut;
        if (c == pv) {
          dsh[pv] = piv;
          rdsh[pv] = r;
        }
        const double wq = bcast(bs, pv);
        if (own && c > pv) bs = fma(-ut, wq, bs);
        if (i < 15) {
#pragma unroll
          for (int m0 = i + 1; m0 < 16; ++m0) a[m0] = fma(-u[m0], ut, a[m0]);
          piv = bcast(a[i + 1], pv + 1);
        }
      }
    } else
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int pv = 16 * J + i;
      double* cb = colbuf + 64 * (i & 1);
      if (c < KP) cb[c] = a[i];  // A[pv][c] (lane pv: the pivot)
      // RLPANEL 2: the one pivot-row entry the NEXT pivot depends on,
      // A[pv][pv + 1], comes by v_readlane (final since the previous pivot),
      // so the LDS round trip of the rest has a whole pivot of slack
      constexpr bool kRl2 = HREC_ALS_RLPANEL == 2;
      const double u1 = (kRl2 && i < 15) ? bcast(a[i], pv + 1) : 0.0;
      // 1 / piv: v_rcp_f64 (~2^-24 relative) + one Newton step
      const double r0 = __builtin_amdgcn_rcp(piv);
      const double r = fma(r0, fma(-piv, r0, 1.0), r0);
      const double ut = a[i] * r;  // Ut[pv][c]
      if (own && c > pv) Up[tri(c) + pv] = ut;
      if (c == pv) {
        dsh[pv] = piv;
        rdsh[pv] = r;
      }
      {
        const double wq = bcast(bs, pv);
        if (own && c > pv) bs = fma(-ut, wq, bs);
      }
      if (i < 15) {
        if constexpr (kRl2) {  // bit-identical: u1 is the value lane pv + 1 stored to cb
          a[i + 1] = fma(-u1, ut, a[i + 1]);
          piv = bcast(a[i + 1], pv + 1);
        } else {
          piv = bcast(fma(-a[i], ut, a[i + 1]), pv + 1);
        }
        wave_lds_sync();
#pragma unroll
        for (int m0 = (i + 1) & ~1; m0 < 16; m0 += 2) {
          const double2 u = *reinterpret_cast<const double2*>(cb + 16 * J + m0);
          if (m0 > i + (kRl2 ? 1 : 0)) a[m0] = fma(-u.x, ut, a[m0]);
          if (!kRl2 || m0 > i) a[m0 + 1] = fma(-u.y, ut, a[m0 + 1]);
        }
      }
    }
    wave_lds_sync();
    // (e) Ut_JK (K > J) back into tile registers, with a D_J-scaled copy;
    // (f) trailing update A_KM -= Ut_JK^T D_J Ut_JM on the f64 matrix cores
    if (J + 1 < NT) {
      double dq[4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) dq[rr] = dsh[16 * J + sub + 4 * rr];
      d4 yv[NT];
#pragma unroll
      for (int K = J + 1; K < NT; ++K) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const double x = Up[tri(16 * K + col) + 16 * J + sub + 4 * rr];
          acc[pidx(J, K)][rr] = x;
          yv[K][rr] = x * dq[rr];
        }
      }
#pragma unroll
      for (int K = J + 1; K < NT; ++K) {
#pragma unroll
        for (int M = K; M < NT; ++M) {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            acc[pidx(K, M)] = __builtin_amdgcn_mfma_f64_16x16x4f64(-acc[pidx(J, K)][rr], yv[M][rr],
                                                                    acc[pidx(K, M)], 0, 0, 0);
        }
      }
    }
  }
  STAMP(3);  // phase 3: factorisation
  const int lc = lane < KP ? lane : KP - 1;
  const double myrd = rdsh[lc];
  if constexpr (HREC_ALS_ABLATE == 3) {  // timing-only: factor without the substitutions
    if (lane < KP) out[lane] = (float)(myrd + Up[tri(lane)]);
    return;
  }
  double bi = bs * myrd;  // v = D^-1 w (w from the panels)
  // back     Ut x = v     (step q: lanes c < q subtract Ut[c][q] * x_q)
#pragma unroll HREC_ALS_SOLVE_UNROLL
  for (int q = KP - 1; q >= 0; --q) {
    const double u = Up[tri(q) + (lane < KP ? lane : 0)];  // Ut[lane][q] for lane < q
    const double xq = bcast(bi, q);
    if (lane < q) bi = fma(-u, xq, bi);
  }
  STAMP(4);  // phase 4: triangular solves
  if (lane < KP) out[NT * (lane & 15) + (lane >> 4)] = (float)bi;
  wave_lds_sync();  // the next row on this wave reuses the LDS slice
}


template <int NT, int CH, int MODE, bool S64 = false>
__device__ __forceinline__ void als_row(int64_t row, int lane, const int64_t* __restrict__ indptr,
                                        const int32_t* __restrict__ indices, const float* __restrict__ values,
                                        const float* __restrict__ src, int64_t n_src, int k, double reg,
                                        float* __restrict__ dst, double* __restrict__ lds) {
  constexpr int KP = 16 * NT;
  const int64_t beg = indptr[row];
  const int64_t end = indptr[row + 1];
  float* __restrict__ out = dst + row * KP;
  if (end == beg) {
    if (lane < KP) out[lane] = 0.f;
    return;
  }
  d4 acc[NT * (NT + 1) / 2];
  double* scratch = lds + RowLds<KP>::kUpPad;
  double* bsh = scratch + 128 + 2 * KP;
  gram_row<NT, CH, MODE, NoHook, S64>(beg, end, lane, indices, values, src, n_src, k, reg, acc, bsh, lds);
  factor_row<NT>(lane, acc, lds, scratch, bsh, out);
}

// One wave per destination row. S64: src points at f64 source factors.
template <int NT, int CH, int MODE, bool S64 = false>
__global__ __launch_bounds__(64, HREC_ALS_WAVES) void als_half_sweep_f64_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ values, int64_t n_rows, const float* __restrict__ src, int64_t n_src,
    int k, double reg, float* __restrict__ dst) {
  __shared__ __attribute__((aligned(16))) double lds[RowLds<16 * NT>::kSize];
  als_row<NT, CH, MODE, S64>(blockIdx.x, threadIdx.x, indptr, indices, values, src, n_src, k, reg, dst, lds);
}

__global__ __launch_bounds__(256) void f32_to_f64_kernel(const float* __restrict__ in, int64_t n,
                                                         double* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = (double)in[i];
}

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
  HREC_REQUIRE(hrec_factor_ld_ok(kp), "als_half_sweep: kp must be 16, 32, 64, 96, 128, 192 or 256 (got %d)", kp);
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
  // the kp-64 gather addresses source rows through one buffer resource, whose
  // 32-bit byte offsets span 4 GiB (16.7M f32 rows of 64)
  HREC_REQUIRE(kp != 64 || n_src * (int64_t)kp * 4 <= (int64_t)0xffffffffll,
               "als_half_sweep: %lld source rows of %d floats exceed the 4 GiB a gather resource spans; shard the "
               "source side", (long long)n_src, kp);
  if (kp > 64) {
    HREC_REQUIRE(accum_mode == 0, "als_half_sweep: kp > 64 supports accum_mode 0 (f64) only");
    return hrec_als_half_sweep_wide(indptr, indices, values, n_rows, src_factors, n_src, k, kp, reg_param,
                                    dst_factors, stream);
  }
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

extern "C" int hrec_f32_to_f64(const float* in, int64_t n, double* out, void* stream) {
  HREC_REQUIRE(n >= 0, "f32_to_f64: negative size");
  if (n == 0) return HREC_OK;
  HREC_REQUIRE(in && out, "f32_to_f64: null pointer");
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(f32_to_f64_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), in, n, out);
  return check_launch("f32_to_f64_kernel");
}

extern "C" int hrec_als_half_sweep_src64(const int64_t* indptr, const int32_t* indices, const float* values,
                                         int64_t n_rows, const double* src64, int64_t n_src, int k, int kp,
                                         double reg_param, float* dst_factors, void* stream) {
  HREC_REQUIRE(kp == 64, "als_half_sweep_src64: kp must be 64 (got %d)", kp);
  HREC_REQUIRE(k >= 1 && k <= kp, "als_half_sweep_src64: need 1 <= k <= kp (k=%d kp=%d)", k, kp);
  HREC_REQUIRE(n_rows >= 0 && n_src >= 0, "als_half_sweep_src64: negative size");
  HREC_REQUIRE(n_rows < 0x7fffffffll && n_src < 0x7fffffffll, "als_half_sweep_src64: too many rows for one launch");
  HREC_REQUIRE(n_src * (int64_t)kp * 8 <= (int64_t)0xffffffffll,
               "als_half_sweep_src64: %lld f64 source rows exceed the 4 GiB a gather resource spans", (long long)n_src);
  HREC_REQUIRE(reg_param >= 0.0, "als_half_sweep_src64: reg_param must be >= 0");
  if (n_rows == 0) return HREC_OK;
  HREC_REQUIRE(indptr && dst_factors, "als_half_sweep_src64: null pointer");
  HREC_REQUIRE(n_src > 0 && src64 && indices && values, "als_half_sweep_src64: null source factors / CSR arrays");
  HREC_REQUIRE(((uintptr_t)src64 & 15) == 0, "als_half_sweep_src64: src64 must be 16-B aligned");
  hipLaunchKernelGGL((als_half_sweep_f64_kernel<4, HREC_ALS_CH0, 0, true>), dim3((unsigned)n_rows), dim3(64), 0,
                     as_stream(stream), indptr, indices, values, n_rows, reinterpret_cast<const float*>(src64), n_src,
                     k, reg_param, dst_factors);
  return check_launch("als_half_sweep_f64_kernel (f64 sources)");
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
