// K9x: the exact hybrid top-k (precision "exact", BASELINE config c2: rank-64
// ALS + d = 64 towers) without writing either [B, N] score matrix — what
// get_hybrid_recommendations does per user (src/hybrid_system.py:95-116: the
// ALS transform's JVM f32 dot + the Keras Dot over every candidate, one
// MinMaxScaler per model, 0.8 / 0.2 fusion, stable sorted()[:top_k]) for a
// batch of users over an item shard, bit for bit the result of
// hrec_als_score + hrec_tt_score + hrec_rows_minmax_f32 + hrec_fuse_rows_topk.
//
// The JVM-exact ALS score (a sequential chain of rounded f32 products and
// sums) cannot run on the matrix cores, and the scaler needs every row's exact
// extremes before any fused score exists. So the scores of every pair are
// first APPROXIMATED on the bf16 matrix cores, with a rigorous error bound,
// and the exact chains run only where the bound cannot decide:
//   phase 1 (hx_stats_kernel): both models' GEMMs on the bf16 matrix cores
//     (v_mfma_f32_32x32x16_bf16, f32 accumulation) in split form: every
//     operand as hi + lo bf16 (x = xh + xl + r, |r| <= 2^-16 |x|) and the
//     score as uh.vh + uh.vl + ul.vh; no score stores: per user and 32-item
//     group the approximate max and min of both models (16 B per user and
//     group);
//   phase 2a (hx_pre_kernel, one block per user):
//     a. exact extremes: |approx - exact| <= E = 2^-13 ||u|| max_j ||v_j||
//        (the dropped terms ul.vl and the split residues: 3 2^-16 sum
//        |u_c v_c|; the f32 accumulation of 3k products and the JVM chain's
//        own rounding: (3k + k) 2^-24 sum |u_c v_c| at k <= 128; twice that
//        margin; sum |u_c v_c| <= ||u|| ||v||), so the item
//        holding a model's exact max lies in a group whose approximate max is
//        within 2E of the approximate extreme (likewise the min). Those groups
//        are rescored exactly: the ALS JVM chain per item, the two-tower score
//        by hrec_dot_scores' own MFMA chain (v_mfma_f32_16x16x4_f32, k order
//        16 ks + 4 g + e) — the same bits as the materialised scores;
//     [with the items sharded, the caller all-reduces the extremes here (C2)]
//     b. per group an upper bound of every fused score in it (hp_fuse of the
//        approximate maxima + E, rounded up to f32: the fusion arithmetic is
//        non-decreasing in both scores); tau = the kk-th best lower bound of
//        a few seed groups' fused scores (each wave's two groups with the
//        largest bounds); every group whose bound reaches tau joins a global
//        queue of group pairs;
//   phase 2b (hx_pairs_kernel, persistent): the waves pull the queued pairs
//     of all users from one counter (a user's live groups vary by an order
//     of magnitude; a block per user waited on the heaviest) and score their
//     items exactly where an item's own bound still reaches tau; those exact
//     fused scores are the user's candidates;
//   phase 2c (hx_final_kernel, one block per user): the stable top-k (ties ->
//     smaller item) of the candidates. An item outside them has a fused
//     score below tau, under kk items already found.
//   Users with non-finite or huge norms, too many live groups or candidates,
//   or whose kk best include a NaN or fewer than kk items, rescore every
//   group in 2c (the order of NaN items is by item id over the whole shard).
#include "common.h"
#include "hybrid_common.h"

namespace hrec {

typedef float hx_f16 __attribute__((ext_vector_type(16)));
typedef __bf16 hx_bf8 __attribute__((ext_vector_type(8)));
__device__ hp_f4 hx_sbuf_load(hrec_rsrc_t rsrc, int vindex, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.struct.buffer.load.v4f32");

union HxFrag {
  int4 i;
  hp_f4 f;
};

constexpr int kHxGrp = 32;       // items per statistics group (one 32-row MFMA tile)
constexpr int kHxMaxK = 8;       // top_k handled here (kFuseK of the materialised path)
constexpr double kHxRel = 0x1p-13;
constexpr double kHxAbs = 1e-30;  // denormal products the matrix cores may flush
constexpr double kHxHuge = 0x1p60;  // a bound above this (or non-finite): rescore every group
constexpr int kHxThreads1 = 256;
constexpr int kHxThreads2 = 512;
constexpr int kHxStatsLds = 8192;  // group records a phase-2 block keeps in LDS (128 KiB)

#ifndef HREC_HX_SCAN_BATCH
#define HREC_HX_SCAN_BATCH 64  // item columns whose loads a full-width DK-64 phase-2 scan issues at once
#endif
#ifndef HREC_HX_NSP_MAX
#define HREC_HX_NSP_MAX 8  // seed pairs scanned beside the extremes' pairs (mode 2), at most
#endif
#ifndef HREC_HX_UB64
// phase-1 users per tile at DK 64: 256 = one 512-thread block per CU (139 KB
// of LDS, 2 waves per SIMD), every item fragment read once per 256-user
// batch (half the item operand reads of 128-user tiles); measured c2 batch
// 0.1022 -> 0.1002 ms
#define HREC_HX_UB64 256
#endif
template <int DK>
struct HxShape {
  static constexpr int KS = DK / 16;               // 32x32x16 k-steps per operand half
  static constexpr int kOpB = DK * 4;              // bytes per operand row: [hi | lo] bf16
  static constexpr int kRowB = kOpB + 16;          // LDS bytes per staged user row
  static constexpr int UB = DK == 64 ? HREC_HX_UB64 : 64;  // users per tile (2 x UB rows of LDS)
  static constexpr int kThreads = UB == 256 ? 512 : kHxThreads1;  // phase-1 block
  static constexpr int kBlocksPerCU = UB == 256 ? 1 : 2;
};

__device__ __forceinline__ float hx_up(double x) {  // the smallest float >= x
  float f = (float)x;
  if ((double)f < x) f = nextafterf(f, INFINITY);
  return f;
}
__device__ __forceinline__ float hx_down(double x) {  // the largest float <= x
  float f = (float)x;
  if ((double)f > x) f = nextafterf(f, -INFINITY);
  return f;
}
__device__ __forceinline__ float hx_u2f(uint32_t u) { return __uint_as_float(u); }

// Split bf16 of x: hi = bf16(x), lo = bf16(x - hi) (x - hi is exact in f32).
__device__ __forceinline__ void hx_split(float x, uint16_t& hi, uint16_t& lo) {
  const uint32_t h = hp_bf16(x);
  hi = (uint16_t)h;
  lo = (uint16_t)hp_bf16(x - __uint_as_float(h << 16));
}

// 0. Split bf16 user operands [2][B][2 DK] ([hi | lo] per row): the ALS rows
// als_users[rows[b]] (a row outside [0, n_rows) reads as NaN, as
// hrec_als_score's unknown users), the two-tower rows; columns >= width zero.
__global__ __launch_bounds__(128) void hx_user_ops_kernel(const float* __restrict__ U, int64_t ldu,
                                                          const int64_t* __restrict__ rows, int64_t n_rows, int ka,
                                                          const float* __restrict__ T, int64_t ldt, int kt, int B,
                                                          int dk, uint16_t* __restrict__ uop, float* __restrict__ uf,
                                                          int* __restrict__ uok, int* __restrict__ flag) {
  const int b = blockIdx.x, m = blockIdx.y;
  if (b == 0 && m == 0 && threadIdx.x < 2) flag[threadIdx.x] = 0;  // the flag + pair total (no reset launch)
  int64_t r = b;
  bool bad = false;
  if (m == 0 && rows) {
    r = rows[b];
    bad = r < 0 || r >= n_rows;
  }
  const float* src = m ? T + (int64_t)b * ldt : U + (bad ? 0 : r) * ldu;
  const int w = m ? kt : ka;
  uint16_t* out = uop + ((int64_t)m * B + b) * 2 * dk;
  float* of = uf + ((int64_t)m * B + b) * dk;  // the f32 row the exact chains read (phase 2)
  for (int c = threadIdx.x; c < dk; c += blockDim.x) {
    float v = 0.f;
    if (c < w) v = bad ? __builtin_nanf("") : src[c];
    hx_split(v, out[c], out[dk + c]);
    of[c] = v;
  }
  if (m == 0 && threadIdx.x == 0) uok[b] = bad ? 0 : 1;
}

// Item-side operands (once per shard): split bf16 rows [2][N][2 dk] (ALS,
// two-tower; [hi | lo], zero beyond the width) and each model's largest row
// 2-norm rounded up (+inf when a row holds a non-finite value or the norm is
// huge). One thread per (row, model); the ALS factors come transposed
// (A[c * lda + row], hrec_als_score's layout), the two-tower rows row-major.
__global__ __launch_bounds__(256) void hx_prepare_kernel(const float* __restrict__ A, int64_t lda, int ka,
                                                         const float* __restrict__ T, int64_t ldt, int kt,
                                                         int64_t N, int dk, uint16_t* __restrict__ out,
                                                         unsigned* __restrict__ norms) {
  const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int m = blockIdx.y;
  double ss = 0.0;
  bool bad = false;
  if (row < N) {
    uint32_t* o = reinterpret_cast<uint32_t*>(out + ((int64_t)m * N + row) * 2 * dk);
    const int w = m ? kt : ka;
    for (int c = 0; c < dk; c += 2) {
      float v[2];
#pragma unroll
      for (int e = 0; e < 2; ++e)
        v[e] = c + e < w ? (m ? T[row * ldt + c + e] : A[(int64_t)(c + e) * lda + row]) : 0.f;
      uint16_t h[2], l[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        hx_split(v[e], h[e], l[e]);
        ss += (double)v[e] * (double)v[e];
        bad = bad || !isfinite(v[e]);
      }
      o[c >> 1] = (uint32_t)h[0] | ((uint32_t)h[1] << 16);
      o[(dk + c) >> 1] = (uint32_t)l[0] | ((uint32_t)l[1] << 16);
    }
  }
  const double nrm = sqrt(ss) * (1.0 + 1e-6);
  unsigned f = __float_as_uint((bad || !(nrm < kHxHuge)) ? INFINITY : hx_up(nrm));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned o = (unsigned)__shfl_xor((int)f, off, kWave);
    f = o > f ? o : f;  // non-negative floats order as their bits
  }
  if ((threadIdx.x & 63) == 0) atomicMax(&norms[m], f);
}

// 1. Phase 1: block = (user tile of UB users, `per` items); each wave walks
// every fourth 32-item slice of them, keeps a slice's item fragments (both models,
// hi and lo, every k-step) in registers and sweeps the tile's users in chunks
// of 32 from LDS; the last chunk refills the fragments with the next slice's.
// MFMA roles: A = items (32 rows), B = users (32 columns), so lane (h, c)
// holds user c and items 8 q + 4 h + r (register 4 q + r). Per (user, group):
// [max, min] of each model's approximate scores (fmaxf / fminf: NaN-free,
// like hrec_rows_minmax_f32), one 16-B record.
#ifdef HREC_HX_STAMPS
__device__ unsigned long long g_hx1_stamps[4096][4];  // per block: start, staged, wave 0 done, wave 3 done
#define HX1_STAMP(i)                                                                         \
  do {                                                                                       \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096) g_hx1_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define HX1_STAMP(i)
#endif

template <int DK>
__global__ __launch_bounds__(HxShape<DK>::kThreads, DK == 64 ? HxShape<DK>::kBlocksPerCU : 1) void hx_stats_kernel(const uint16_t* __restrict__ uop, int B, int n_ut,
                                                               const char* __restrict__ items, int64_t N, int G,
                                                               int64_t per, float* __restrict__ stats) {
  using S = HxShape<DK>;
  constexpr int KS = S::KS, UB = S::UB, kRowB = S::kRowB, kOpB = S::kOpB, T1 = S::kThreads;
  __shared__ __attribute__((aligned(16))) char us[2 * UB * kRowB];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int ut = (int)(blockIdx.x % (unsigned)n_ut);
  const int64_t i0 = (int64_t)(blockIdx.x / (unsigned)n_ut) * per;  // per: a multiple of 32
  const int64_t i1 = i0 + per < N ? i0 + per : N;
  const int b0 = ut * UB;
  const int ub = B - b0 < UB ? B - b0 : UB;
  const char* ia = items;                        // ALS operand [N][2 DK]
  const char* it = items + (size_t)N * kOpB;     // two-tower operand [N][2 DK]
  const hrec_rsrc_t ra = rows_rsrc(ia, i0, kOpB, N), rt = rows_rsrc(it, i0, kOpB, N);
  // DK 64: two fragment sets (double buffer): the next slice's item
  // fragments load at the start of this slice, so their latency hides behind
  // its 4 user chunks (loading them at the last chunk left one HBM round trip
  // per slice exposed: 42k loop ticks per wave for 20k of MFMA work per SIMD);
  // 244 VGPRs keep 2 waves per SIMD. DK 128 (its fragments twice the size):
  // one set, refilled after the last chunk.
  constexpr bool kDB = DK == 64;
  HxFrag fa0[2][KS], ft0[2][KS], fa1[2][KS], ft1[2][KS];  // [hi / lo][k-step]
  auto load = [&](int64_t jb, HxFrag (&fa)[2][KS], HxFrag (&ft)[2][KS]) {
    const int64_t j = jb + c;
    const int vi = j < N ? (int)(j - i0) : 0x7fffffff;  // out of range: the buffer check reads zeros
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        fa[p][ks].f = hx_sbuf_load(ra, vi, p * (DK * 2) + 32 * ks + 16 * h, 0, 0);
        ft[p][ks].f = hx_sbuf_load(rt, vi, p * (DK * 2) + 32 * ks + 16 * h, 0, 0);
      }
  };
  int64_t jb = i0 + 32 * w;
  if (w == 0) HX1_STAMP(0);
  if (jb < i1) load(jb, fa0, ft0);  // the first slice arrives while the users are staged
  // users -> LDS: every load of a thread in flight before its stores (one
  // round trip, not one per 16-B chunk)
  constexpr int CPR = kOpB / 16;  // 16-B chunks per user row
  constexpr int kPer = 2 * UB * CPR / T1;
  static_assert(kPer * T1 == 2 * UB * CPR, "whole chunks per thread");
  {
    int4 v[kPer];
#pragma unroll
    for (int e = 0; e < kPer; ++e) {
      const int o = threadIdx.x + e * T1;
      const int m = o / (UB * CPR), rem = o % (UB * CPR), r = rem / CPR, q = rem % CPR;
      v[e] = int4{0, 0, 0, 0};
      if (r < ub) v[e] = *reinterpret_cast<const int4*>(uop + (int64_t)(m * B + b0 + r) * (2 * DK) + 8 * q);
    }
#pragma unroll
    for (int e = 0; e < kPer; ++e) {
      const int o = threadIdx.x + e * T1;
      const int m = o / (UB * CPR), rem = o % (UB * CPR), r = rem / CPR, q = rem % CPR;
      *reinterpret_cast<int4*>(us + (m * UB + r) * kRowB + 16 * q) = v[e];
    }
  }
  __syncthreads();
  if (w == 0) HX1_STAMP(1);
  // one 32-item slice with the fragments in (fa, ft); the next slice's
  // fragments go to (na, nt) first. Returns false after the range's last slice.
  auto slice = [&](HxFrag (&fa)[2][KS], HxFrag (&ft)[2][KS], HxFrag (&na)[2][KS], HxFrag (&nt)[2][KS]) {
    const bool full = jb + 32 <= N;
    const int64_t jn = jb + 32 * (T1 / 64);
    const bool more = jn < i1;
    if (kDB && more) load(jn, na, nt);
    for (int ch = 0; 32 * ch < ub; ++ch) {
      hx_f16 acc[2];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[m][v] = 0.f;
      const char* ura = us + (32 * ch + c) * kRowB + 16 * h;
      const char* urt = us + (UB + 32 * ch + c) * kRowB + 16 * h;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        HxFrag ah, al, th, tl;
        ah.i = *reinterpret_cast<const int4*>(ura + 32 * ks);
        al.i = *reinterpret_cast<const int4*>(ura + DK * 2 + 32 * ks);
        th.i = *reinterpret_cast<const int4*>(urt + 32 * ks);
        tl.i = *reinterpret_cast<const int4*>(urt + DK * 2 + 32 * ks);
#define HX_MMA(ACC, X, Y) \
  ACC = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(hx_bf8, (X).i), __builtin_bit_cast(hx_bf8, (Y).i), ACC, 0, 0, 0)
        HX_MMA(acc[0], fa[0][ks], ah);  // vh.uh
        HX_MMA(acc[1], ft[0][ks], th);
        HX_MMA(acc[0], fa[1][ks], ah);  // vl.uh
        HX_MMA(acc[1], ft[1][ks], th);
        HX_MMA(acc[0], fa[0][ks], al);  // vh.ul
        HX_MMA(acc[1], ft[0][ks], tl);
#undef HX_MMA
      }
      float mx[2], mn[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        float hi = -INFINITY, lo = INFINITY;
        if (full) {
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            hi = fmaxf(hi, acc[m][v]);
            lo = fminf(lo, acc[m][v]);
          }
        } else {
#pragma unroll
          for (int v = 0; v < 16; ++v)
            if (jb + 8 * (v >> 2) + 4 * h + (v & 3) < N) {
              hi = fmaxf(hi, acc[m][v]);
              lo = fminf(lo, acc[m][v]);
            }
        }
        mx[m] = hi;
        mn[m] = lo;
      }
      // the two lane halves hold the two halves of the group: one
      // v_permlane32_swap per register pair folds them for both models
      const auto X = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx[0]), __float_as_uint(mx[1]), false, false);
      const auto Y = __builtin_amdgcn_permlane32_swap(__float_as_uint(mn[0]), __float_as_uint(mn[1]), false, false);
      const float hi = fmaxf(hx_u2f(X[0]), hx_u2f(X[1]));  // lanes < 32: ALS, lanes >= 32: two-tower
      const float lo = fminf(hx_u2f(Y[0]), hx_u2f(Y[1]));
      const int b = b0 + 32 * ch + c;
      if (!kDB && more && 32 * (ch + 1) >= ub) load(jn, na, nt);  // last chunk: the next slice's fragments
      if (b < B) *reinterpret_cast<float2*>(stats + ((int64_t)b * G + (jb >> 5)) * 4 + 2 * h) = make_float2(hi, lo);
    }
    jb = jn;
    return more;
  };
  if (jb < i1) {  // wave-uniform; no barrier follows
    if constexpr (kDB) {
      while (slice(fa0, ft0, fa1, ft1) && slice(fa1, ft1, fa0, ft0)) {
      }
    } else {
      while (slice(fa0, ft0, fa0, ft0)) {
      }
    }
  }
  if (w == 0) HX1_STAMP(2);
  if (w == 3) HX1_STAMP(3);
}

#ifdef HREC_HX_STAMPS
// Diagnostic builds only: per block (thread 0) s_memtime at the phase points
// of hx_pre_kernel, plain vector stores.
constexpr int kHxStampBlocks = 1024;
__device__ unsigned long long g_hx_stamps[kHxStampBlocks][16];
#define HX_STAMP(i)                                                            \
  do {                                                                         \
    if (tid == 0 && b < kHxStampBlocks) g_hx_stamps[b][i] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define HX_STAMP(i)
#endif

// Per-user state phase 2a hands to 2b / 2c.
struct HxRec {
  double tau;          // the bound an item's fused bound must reach to be scored exactly
  double ascale, amin_;
  double Ef;           // |two-tower fma chain - exact| bound
  float tscale, tmin_;
  int state;           // kHxQueued / kHxEvery / kHxNaN
  int pair_base;       // the user's pairs: [pair_base, pair_base + n_pairs) of the queue
  int n_pairs;
  int pad;
};
constexpr int kHxQueued = 0;  // live pairs queued for 2b, candidates ranked in 2c
constexpr int kHxEvery = 1;   // no usable bound: 2c scores every group
constexpr int kHxNaN = 2;     // a model without any number: every fused score NaN
constexpr int kHxSlots = 8;  // a pair's best exact candidates kept (>= top_k)
// the live-group list in 2a's LDS holds 2 x this many groups (a quarter of
// the shard's groups within [512, 8192]); the queue holds B x this many pairs
// (a user with more live groups writes them window by window; a user the
// queue has no room for: kHxEvery)
__host__ __device__ inline int hx_pair_cap(int G) { return G / 8 < 512 ? 512 : (G / 8 > 8192 ? 8192 : G / 8); }
struct HxArgs {
  int ka, kt, B;
  const float* Vat;  // ALS item factors transposed: item j, column c at Vat[c * lda + j]
  int64_t lda;
  const float* Vt;   // two-tower item vectors [N] (row-major, row stride ldv)
  int64_t ldv;
  const float* Vtt;  // the same transposed: Vtt[c * ldtt + j]
  int64_t ldtt;
  const float* inorm;  // [2] the item operands' largest norms (hx_prepare_kernel)
  const float* uf;     // [2][B][DK] the batch's f32 user rows (hx_user_ops_kernel)
  const int* uok;      // [B] ALS row known
  int64_t N;
  int G;
  const float* stats;  // [B][G][4] phase 1
  float* mm_a;         // [2][B] ALS [min; max] (written by modes 0 / 2, read by mode 1)
  float* mm_t;         // [2][B] two-tower
  double w0, w1;
  int kk;
  int64_t idx_offset;
  int64_t* out_idx;
  double* out_val;
  int* counts;  // [2][B]: groups rescored for the extremes / queued for the top-k
  int* flag;    // set when a user rescored every group
  HxRec* rec;   // [B]
  int pair_cap;
  int pair_capacity;  // B * pair_cap: the queue's entries
  int4* pairs;  // [B * pair_cap] (user, group A, group B)
  int* pair_total;
  double* cv;   // [pair][kHxSlots] a pair's best exact fused scores
  int64_t* ci;  // [pair][kHxSlots] their items
  int* pc;      // [pair] how many
};

// Shared by the phase-2 kernels (one wave, lane l = item l of a pair of
// 32-item groups). The ALS score is the JVM chain itself, read from the
// TRANSPOSED item factors (per column one coalesced 128-B run per group;
// row-major gathers touched 64 lines per load instruction). The two-tower
// score is first bounded by an f32 fma chain over the transposed item
// vectors (within Ef of the exact score); the exact two-tower score —
// hrec_dot_scores' MFMA chain over row-major rows — only for the items whose
// bound can still matter, 16 per MFMA round.
template <int DK, bool FULL>
struct HxWave {
  const HxArgs& a;
  const float* sua;  // the user's f32 rows in LDS
  const float* sut;
  int ka, kt, lane;

  __device__ __forceinline__ bool item_of(int gA, int gB, int64_t& j) const {
    const int gl = lane < 32 ? gA : gB;
    j = (int64_t)gl * kHxGrp + (lane & 31);
    return gl >= 0 && j < a.N;
  }
  // exact ALS score (sequential rounded products and sums over c < ka,
  // Spark's dotProduct += a(i) * b(i)) and the two-tower fma chain of item j:
  // 32 columns of both per batch of loads
  __device__ __forceinline__ void scan(int64_t j, bool ok, float& s_als, float& t_fma) const {
#pragma clang fp contract(off)
    const int64_t jj = ok ? j : 0;
    const float* pa = a.Vat + jj;
    const float* pt = a.Vtt + jj;
    const int n = ka > kt ? ka : kt;
    // columns per batch of loads: all 64 at once for full-width DK 64 (one
    // memory round trip per scan instead of two: c2 batch 0.1025 -> 0.0984 ms,
    // 2b 26.1 -> 23.2 us); 32 elsewhere (64 spills in hx_pre's DK 128 / partial
    // width kernels)
    constexpr int NB = (FULL && DK == 64) ? HREC_HX_SCAN_BATCH : 32;
    float s = 0.f, t = 0.f;
    for (int c0 = 0; c0 < n; c0 += NB) {
      float va[NB], vt[NB];
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        va[q] = (FULL || c0 + q < ka) ? pa[(int64_t)(c0 + q) * a.lda] : 0.f;
        vt[q] = (FULL || c0 + q < kt) ? pt[(int64_t)(c0 + q) * a.ldtt] : 0.f;
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < NB; q += 4) {
        const float4 u = *reinterpret_cast<const float4*>(sua + c0 + q);
        const float4 w = *reinterpret_cast<const float4*>(sut + c0 + q);
        float p = u.x * va[q];
        s = s + p;
        p = u.y * va[q + 1];
        s = s + p;
        p = u.z * va[q + 2];
        s = s + p;
        p = u.w * va[q + 3];
        s = s + p;  // columns >= ka: 0 * 0, adds +0 (a no-op)
        t = fmaf(w.x, vt[q], t);
        t = fmaf(w.y, vt[q + 1], t);
        t = fmaf(w.z, vt[q + 2], t);
        t = fmaf(w.w, vt[q + 3], t);
      }
    }
    s_als = s;
    t_fma = t;
  }
  // exact two-tower scores of up to 16 items (A = their rows, row cc = the
  // item of lane cc; lane (g, cc < 4) gets item 4 g + cc)
  __device__ __forceinline__ float tt_exact16(int64_t jrow, bool has) const {
    const int g4 = lane >> 4;
    const float* row = a.Vt + (has ? jrow : 0) * a.ldv + 4 * g4;
    const int KT = kt >> 4;
    hp_f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int ks0 = 0; ks0 < KT; ks0 += 4) {
      HxFrag itf[4];
#pragma unroll
      for (int kq = 0; kq < 4; ++kq)
        itf[kq].f = (FULL || ks0 + kq < KT) ? *reinterpret_cast<const hp_f4*>(row + 16 * (ks0 + kq))
                                            : hp_f4{0.f, 0.f, 0.f, 0.f};
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kq = 0; kq < 4; ++kq) {
        if (FULL || ks0 + kq < KT) {
          HxFrag uf;
          uf.f = *reinterpret_cast<const hp_f4*>(sut + 16 * (ks0 + kq) + 4 * g4);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(itf[kq].f[e], uf.f[e], acc, 0, 0, 0);
        }
      }
    }
    return hp_pick(acc, lane & 3);
  }
  // every lane with m's bit set, 16 per round: fn(j, s_als, t_exact, bit) on
  // lane (g, cc < 4) for the round's item 4 g + cc, the item of lane `bit`
  // (wave-uniform)
  template <class F>
  __device__ __forceinline__ void exact_rounds(uint64_t m, int64_t j, float s_als, F fn) const {
    const int cc = lane & 15;
    while (m) {
      int my = -1;
      for (int i = 0; i < 16 && m; ++i) {
        const int bit = __builtin_ctzll(m);
        m &= m - 1;
        my = cc == i ? bit : my;
      }
      const int src = my < 0 ? 0 : my;
      const int64_t jr = __shfl(j, src, kWave);
      const float ar = __shfl(s_als, src, kWave);
      const float tx = tt_exact16(jr, my >= 0);
      const int q = 4 * (lane >> 4) + (cc & 3);
      const int myq = __shfl(my, q, kWave);
      const int64_t jq = __shfl(jr, q, kWave);
      const float aq = __shfl(ar, q, kWave);
      if (cc < 4 && myq >= 0) fn(jq, aq, tx, myq);
    }
  }
};

// fminf / fmaxf over the block (512 threads), 4 values
__device__ __forceinline__ void hx_block_minmax(float& lo_a, float& hi_a, float& lo_t, float& hi_t,
                                                float (*sred)[4], int lane, int wv) {
  lo_a = fminf(lo_a, hp_dpp32<0xB1>(lo_a)), hi_a = fmaxf(hi_a, hp_dpp32<0xB1>(hi_a));
  lo_t = fminf(lo_t, hp_dpp32<0xB1>(lo_t)), hi_t = fmaxf(hi_t, hp_dpp32<0xB1>(hi_t));
  lo_a = fminf(lo_a, hp_dpp32<0x4E>(lo_a)), hi_a = fmaxf(hi_a, hp_dpp32<0x4E>(hi_a));
  lo_t = fminf(lo_t, hp_dpp32<0x4E>(lo_t)), hi_t = fmaxf(hi_t, hp_dpp32<0x4E>(hi_t));
  lo_a = fminf(lo_a, hp_dpp32<0x141>(lo_a)), hi_a = fmaxf(hi_a, hp_dpp32<0x141>(hi_a));
  lo_t = fminf(lo_t, hp_dpp32<0x141>(lo_t)), hi_t = fmaxf(hi_t, hp_dpp32<0x141>(hi_t));
  lo_a = fminf(lo_a, hp_dpp32<0x140>(lo_a)), hi_a = fmaxf(hi_a, hp_dpp32<0x140>(hi_a));
  lo_t = fminf(lo_t, hp_dpp32<0x140>(lo_t)), hi_t = fmaxf(hi_t, hp_dpp32<0x140>(hi_t));
  lo_a = fminf(lo_a, hp_xor16(lo_a)), hi_a = fmaxf(hi_a, hp_xor16(hi_a));
  lo_t = fminf(lo_t, hp_xor16(lo_t)), hi_t = fmaxf(hi_t, hp_xor16(hi_t));
  lo_a = fminf(lo_a, hp_xor32(lo_a)), hi_a = fmaxf(hi_a, hp_xor32(hi_a));
  lo_t = fminf(lo_t, hp_xor32(lo_t)), hi_t = fmaxf(hi_t, hp_xor32(hi_t));
  __syncthreads();  // sred's previous readers are done
  if (lane == 0) sred[wv][0] = lo_a, sred[wv][1] = hi_a, sred[wv][2] = lo_t, sred[wv][3] = hi_t;
  __syncthreads();
  lo_a = sred[0][0], hi_a = sred[0][1], lo_t = sred[0][2], hi_t = sred[0][3];
#pragma unroll
  for (int q = 1; q < 8; ++q) {
    lo_a = fminf(lo_a, sred[q][0]), hi_a = fmaxf(hi_a, sred[q][1]);
    lo_t = fminf(lo_t, sred[q][2]), hi_t = fmaxf(hi_t, sred[q][3]);
  }
}

// The block's kk best of the given entries (each lane's HpList, or n LDS
// entries) by ranking in LDS. Returns 1 (block-uniform) when a NaN or a
// missing entry is among the kk; writes the outputs when out_idx != nullptr
// and the kk-th value to *tau.
struct HxMergeLds {
  uint64_t mk[512];
  int64_t mi[512];
  double mv[512];
  int n, bad;
  double tau;
};
template <int KK>
__device__ int hx_merge(HpList<KK>& L, bool from_lists, HxMergeLds& M, double* rv, int64_t* ri, int kk, int lane,
                        int wv, int tid, int64_t b, int64_t idx_offset, int64_t* out_idx, double* out_val) {
  if (from_lists) {
    if (tid == 0) M.n = 0;
    __syncthreads();
    // a wave holding more than 8 entries sends only its kk best (the
    // block's kk best are among the waves' kk best): <= 64 entries to rank
    int wn = 0;
#pragma unroll
    for (int e = 0; e < KK; ++e) wn += __popcll(__ballot(L.i[e] != INT64_MAX));
    if (wn > 8) {  // wave-uniform
      L.wave_top(kk, lane, rv + wv * KK, ri + wv * KK);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // lane 0's LDS writes -> the wave's reads
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lane < kk && ri[wv * KK + lane] != INT64_MAX) {
        const int p = atomicAdd(&M.n, 1);
        const double v = rv[wv * KK + lane];
        const int64_t i = ri[wv * KK + lane];
        M.mk[p] = hp_order_key(v, i), M.mi[p] = i, M.mv[p] = v;
      }
    } else {
#pragma unroll
      for (int e = 0; e < KK; ++e) {
        if (L.i[e] != INT64_MAX) {
          const int p = atomicAdd(&M.n, 1);
          M.mk[p] = hp_order_key(L.v[e], L.i[e]), M.mi[p] = L.i[e], M.mv[p] = L.v[e];
        }
      }
    }
  }
  if (tid == 0) M.bad = 0, M.tau = -INFINITY;
  __syncthreads();
  const int n = M.n;
  if (tid < kk && tid >= n) {  // fewer than kk entries: the missing ranks
    M.bad = 1;
    if (out_idx) {
      out_idx[b * kk + tid] = -1;
      out_val[b * kk + tid] = 0.0;
    }
  }
  for (int q = tid; q < n; q += kHxThreads2) {
    const uint64_t kq = M.mk[q];
    const int64_t iq = M.mi[q];
    int rank = 0;
    for (int x = 0; x < n; ++x) {
      const uint64_t kx = M.mk[x];
      rank += (int)(kx > kq) | ((int)(kx == kq) & (int)(M.mi[x] < iq));
    }
    if (rank < kk) {
      const double vq = M.mv[q];
      if (vq != vq) M.bad = 1;
      if (out_idx) {
        out_idx[b * kk + rank] = iq + idx_offset;
        out_val[b * kk + rank] = vq;
      }
      if (rank == kk - 1) M.tau = vq;
    }
  }
  __syncthreads();
  return M.bad;
}

// 2a. One 512-thread block per user. MODE 0: the exact extremes only
// (mm_a / mm_t out); 1: with the given (global) extremes, the top-k
// prologue; 2: both (one shard). Prologue: tau from seed groups, then every
// live pair (group bound >= tau) into the global queue for 2b.
template <int DK, int MODE, bool FULL>
__global__ __launch_bounds__(kHxThreads2) void hx_pre_kernel(HxArgs a) {
#pragma clang fp contract(off)
  constexpr int KK = kHxMaxK;
  static_assert(8 * KK == 64, "one merge slot per lane of wave 0");
  constexpr int kList = 1024;  // groups compacted per sweep window
  __shared__ __attribute__((aligned(16))) float sua[DK];
  __shared__ __attribute__((aligned(16))) float sut[DK];
  __shared__ float sred[8][4];
  __shared__ double se[3];
  __shared__ double rv[8 * KK];
  __shared__ int64_t ri[8 * KK];
  __shared__ int s_cnt, s_n;
  __shared__ int s_list[kList];
  __shared__ HxMergeLds M;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int b = blockIdx.x;
  const int G = a.G;
  const int ka = FULL ? DK : a.ka, kt = FULL ? DK : a.kt;
  // the user's group records: staged in LDS once when they fit (the passes
  // below read them several times), else read from memory
  extern __shared__ __attribute__((aligned(16))) float4 st_lds[];
  const float4* st_glob = reinterpret_cast<const float4*>(a.stats) + (int64_t)b * G;
  const bool st_in_lds = G <= kHxStatsLds;
  const float4* st_row = st_in_lds ? st_lds : st_glob;
  int* s_glist = reinterpret_cast<int*>(st_lds + (st_in_lds ? G : 0));  // [2 pair_cap] the live groups
  HX_STAMP(0);
  // the user rows first, then the group records (LDS when they fit) with the
  // approximate extremes folded into the same pass
  float ur_a = 0.f, ur_t = 0.f;
  if (tid < DK) {
    ur_a = a.uf[(int64_t)b * DK + tid];
    ur_t = a.uf[((int64_t)a.B + b) * DK + tid];
  }
  const bool rok = a.uok[b] != 0;
  float AMN = INFINITY, AMX = -INFINITY, TMN = INFINITY, TMX = -INFINITY;
  for (int g0 = tid; g0 < G; g0 += 8 * kHxThreads2) {
    float4 x[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int g = g0 + e * kHxThreads2;
      if (g < G) x[e] = st_glob[g];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int g = g0 + e * kHxThreads2;
      if (g < G) {
        if (st_in_lds) st_lds[g] = x[e];
        AMX = fmaxf(AMX, x[e].x), AMN = fminf(AMN, x[e].y), TMX = fmaxf(TMX, x[e].z), TMN = fminf(TMN, x[e].w);
      }
    }
  }
  if (tid < DK) sua[tid] = ur_a, sut[tid] = ur_t;
  if (tid == 0) s_cnt = 0, s_n = 0;
  __syncthreads();
  if (wv == 0) {  // the bounds of both models (f64 norms)
    double sa = 0.0, sb = 0.0;
    for (int c = lane; c < DK; c += 64) {
      sa += (double)sua[c] * (double)sua[c];
      sb += (double)sut[c] * (double)sut[c];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      sa += __shfl_xor(sa, off, kWave);
      sb += __shfl_xor(sb, off, kWave);
    }
    if (lane == 0) {
      se[0] = kHxRel * (sqrt(sa) * (1.0 + 1e-6)) * (double)a.inorm[0] + kHxAbs;
      se[1] = kHxRel * (sqrt(sb) * (1.0 + 1e-6)) * (double)a.inorm[1] + kHxAbs;
      // the f32 fma chain vs the MFMA chain (bitwise an fma chain): both
      // within gamma_kt sum |u_c v_c| of the real dot
      se[2] = (2.0 * kt + 4.0) * 0x1p-24 * (sqrt(sb) * (1.0 + 1e-6)) * (double)a.inorm[1] + kHxAbs;
    }
  }
  if constexpr (MODE != 1) hx_block_minmax(AMN, AMX, TMN, TMX, sred, lane, wv);  // its barriers publish se
  else __syncthreads();
  HX_STAMP(1);
  const double Ea = se[0], Et = se[1], Ef = se[2];
  const bool bad_a = !(Ea < kHxHuge), bad_t = !(Et < kHxHuge);  // NaN / inf / huge: no bound
  const HxWave<DK, FULL> W{a, sua, sut, ka, kt, lane};
  const double w0 = a.w0, w1 = a.w1;
  const int cap2 = 2 * a.pair_cap;
  // every group with pred(g), in windows of kList groups: compacted into LDS
  // (any order: the results do not depend on it), then dealt to the waves
  // two at a time, round robin (the fallback when the list overflows)
  auto sweep = [&](auto pred, auto pair) {
    for (int g0 = 0; g0 < G; g0 += kList) {
      const int g1 = G - g0 < kList ? G : g0 + kList;
      if (tid == 0) s_n = 0;
      __syncthreads();
      for (int g = g0 + tid; g < g1; g += kHxThreads2)
        if (pred(g)) s_list[atomicAdd(&s_n, 1)] = g;
      __syncthreads();
      const int n = s_n;
      if (tid == 0) s_cnt += n;
      for (int p = wv; 2 * p < n; p += 8) pair(s_list[2 * p], 2 * p + 1 < n ? s_list[2 * p + 1] : -1);
      __syncthreads();  // the list is rewritten by the next window
    }
  };

  // the seeds (top-k modes): each wave's two groups with the largest fused
  // bounds (mode 2: under the scaler of the APPROXIMATE extremes — any choice
  // of seeds is sound, their exact scores bound tau from below); the best
  // 2 nsp of those 16 are scanned in the same round as the extremes' groups
  // (nsp pairs beside them, 4..8, so that no wave scans twice when the
  // extremes need few pairs); a seed's lower bound needs the exact scaler,
  // after the extremes
  constexpr bool kSeeds = MODE != 0;
  __shared__ double s_sv[16];
  __shared__ int s_sg[16];
  HpScale sc0{};
  if constexpr (MODE == 2) sc0 = hp_scale(AMN, AMX, TMN, TMX);
  if constexpr (MODE == 1) sc0 = hp_scale(a.mm_a[b], a.mm_a[a.B + b], a.mm_t[b], a.mm_t[a.B + b]);
  if constexpr (kSeeds) {
    double bu = -INFINITY;
    int64_t bg = INT64_MAX;
    for (int g = 64 * wv + lane; g < G; g += 64 * 8) {
      const float4 x = st_row[g];
      const double u = hp_fuse(sc0, hx_up((double)x.x + Ea), hx_up((double)x.z + Et), w0, w1);
      if (bg == INT64_MAX || hp_better(u, g, bu, bg)) {
        bu = u;
        bg = g;
      }
    }
    double v1 = bu;
    int64_t g1 = bg;
    hp_wave_best(v1, g1);
    if (g1 != INT64_MAX && bg == g1) bg = INT64_MAX;  // the owner drops it
    double v2 = bu;
    int64_t g2 = bg;
    hp_wave_best(v2, g2);
    if (lane == 0) {
      s_sv[2 * wv] = v1, s_sg[2 * wv] = g1 == INT64_MAX ? -1 : (int)g1;
      s_sv[2 * wv + 1] = v2, s_sg[2 * wv + 1] = g2 == INT64_MAX ? -1 : (int)g2;
    }
  }
  float s_sa = 0.f, s_tf = 0.f;  // this wave's seed pair: exact ALS score, fma chain
  int64_t s_j = 0;
  bool s_ok = false;
  // seed pair q: the entries ranked 2q, 2q + 1 of the 16 (lanes 0..15 rank
  // one entry each; better bound first, ties -> the smaller group)
  auto seed_scan = [&](int q) {
    int rank = 99, gl = -1;
    if (lane < 16) {
      gl = s_sg[lane];
      const double v = s_sv[lane];
      int r = 0;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int ge = s_sg[e];
        r += ge >= 0 && ge != gl && hp_better(s_sv[e], ge, v, gl);
      }
      rank = gl >= 0 ? r : 99;
    }
    const uint64_t mA = __ballot(rank == 2 * q), mB = __ballot(rank == 2 * q + 1);
    const int gA = mA ? __shfl(gl, __builtin_ctzll(mA), kWave) : -1;
    const int gB = mB ? __shfl(gl, __builtin_ctzll(mB), kWave) : -1;
    s_ok = W.item_of(gA, gB, s_j);
    W.scan(s_j, s_ok, s_sa, s_tf);
  };

  float amin = INFINITY, amax = -INFINITY, tmin = INFINITY, tmax = -INFINITY;
  if constexpr (MODE != 1) {
    // a. the groups that can hold an exact extreme
    const bool all_a = rok && bad_a, all_t = bad_t;
    const bool use_a = rok && !bad_a && AMX >= AMN, use_t = !bad_t && TMX >= TMN;
    const float a_hi = use_a ? hx_down((double)AMX - 2.0 * Ea) : INFINITY;
    const float a_lo = use_a ? hx_up((double)AMN + 2.0 * Ea) : -INFINITY;
    const float t_hi = use_t ? hx_down((double)TMX - 2.0 * Et) : INFINITY;
    const float t_lo = use_t ? hx_up((double)TMN + 2.0 * Et) : -INFINITY;
    const bool every = all_a || all_t;
    if (every && tid == 0) *a.flag = 1;
    auto pred = [&](int g) {
      if (every) return true;
      const float4 x = st_row[g];
      return x.x >= a_hi || x.y <= a_lo || x.z >= t_hi || x.w <= t_lo;
    };
    float lo_a = INFINITY, hi_a = -INFINITY, lo_t = INFINITY, hi_t = -INFINITY;
    auto pair = [&](int gA, int gB) {
      // exact ALS scores of every item; the exact two-tower score only
      // where the fma chain cannot rule the item out as the pair's
      // extreme (|t_fma - t| <= Ef: the item holding the exact max has
      // t_fma + Ef >= the pair's max of t_fma - Ef, likewise the min)
      int64_t j;
      const bool ok = W.item_of(gA, gB, j);
      float sa, tf;
      W.scan(j, ok, sa, tf);
      if (ok) lo_a = fminf(lo_a, sa), hi_a = fmaxf(hi_a, sa);
      float pm = ok ? tf : -INFINITY, pn = ok ? tf : INFINITY;
      pm = fmaxf(pm, hp_dpp32<0xB1>(pm)), pn = fminf(pn, hp_dpp32<0xB1>(pn));
      pm = fmaxf(pm, hp_dpp32<0x4E>(pm)), pn = fminf(pn, hp_dpp32<0x4E>(pn));
      pm = fmaxf(pm, hp_dpp32<0x141>(pm)), pn = fminf(pn, hp_dpp32<0x141>(pn));
      pm = fmaxf(pm, hp_dpp32<0x140>(pm)), pn = fminf(pn, hp_dpp32<0x140>(pn));
      pm = fmaxf(pm, hp_xor16(pm)), pn = fminf(pn, hp_xor16(pn));
      pm = fmaxf(pm, hp_xor32(pm)), pn = fminf(pn, hp_xor32(pn));
      const bool cand = ok && (every || (double)tf + Ef >= (double)pm - Ef || (double)tf - Ef <= (double)pn + Ef ||
                               tf != tf);
      W.exact_rounds(__ballot(cand), j, sa, [&](int64_t, float, float tx, int) {
        lo_t = fminf(lo_t, tx), hi_t = fmaxf(hi_t, tx);
      });
    };
    // one pass into the LDS list (the windowed sweep when it overflows)
    for (int g = tid; g < G; g += kHxThreads2) {
      if (pred(g)) {
        const int q = atomicAdd(&s_n, 1);
        if (q < cap2) s_glist[q] = g;
      }
    }
    __syncthreads();
    const int n = s_n;
    if (n <= cap2) {
      // work items: the seed pairs (waves 0..nsp-1), then the extremes' pairs
      const int n_ext = (n + 1) / 2;
      const int nsp0 = kSeeds ? (n_ext >= 4 ? 4 : 8 - n_ext) : 0;
      const int nsp = nsp0 < HREC_HX_NSP_MAX ? nsp0 : HREC_HX_NSP_MAX;
      for (int it = wv; it < nsp + n_ext; it += 8) {
        if (it < nsp) {
          seed_scan(it);
        } else {
          const int q = it - nsp;
          pair(s_glist[2 * q], 2 * q + 1 < n ? s_glist[2 * q + 1] : -1);
        }
      }
      if (tid == 0) s_cnt = n;
    } else {
      sweep(pred, pair);
      if (kSeeds) seed_scan(wv);
    }
    hx_block_minmax(lo_a, hi_a, lo_t, hi_t, sred, lane, wv);
    HX_STAMP(2);
    amin = lo_a, amax = hi_a, tmin = lo_t, tmax = hi_t;
    if (tid == 0) {
      a.counts[b] = s_cnt;
      a.mm_a[b] = amin, a.mm_a[a.B + b] = amax;
      a.mm_t[b] = tmin, a.mm_t[a.B + b] = tmax;
    }
    if constexpr (MODE == 0) return;
  } else {
    amin = a.mm_a[b], amax = a.mm_a[a.B + b], tmin = a.mm_t[b], tmax = a.mm_t[a.B + b];
    __syncthreads();  // the seed candidates
    seed_scan(wv);
  }
  // b. the top-k prologue
  HxRec r{};
  r.Ef = Ef;
  if (!(amin <= amax) || !(tmin <= tmax)) {  // every fused score NaN
    if (tid == 0) {
      r.state = kHxNaN;
      a.rec[b] = r;
      a.counts[a.B + b] = 0;
    }
    return;
  }
  const HpScale sc = hp_scale(amin, amax, tmin, tmax);
  r.ascale = sc.ascale, r.amin_ = sc.amin_, r.tscale = sc.tscale, r.tmin_ = sc.tmin_;
  const int kk = a.kk;
  if (bad_a || bad_t || !(isfinite(amin) && isfinite(amax) && isfinite(tmin) && isfinite(tmax))) {
    if (tid == 0) {  // no usable bound: 2c scores every group
      r.state = kHxEvery;
      r.tau = -INFINITY;
      a.rec[b] = r;
      a.counts[a.B + b] = G;
      *a.flag = 1;
    }
    return;
  }
  auto ub_of = [&](int g) {
    const float4 x = st_row[g];
    return hp_fuse(sc, hx_up((double)x.x + Ea), hx_up((double)x.z + Et), w0, w1);
  };
  // tau: a seed's fused score is bounded below by its exact ALS score and its
  // fma chain - Ef, so the kk-th best of those bounds (distinct items) is a
  // lower bound of the shard's kk-th best fused score
  HpList<KK> L;
  L.reset();
  if (s_ok) L.insert(hp_fuse(sc, s_sa, hx_down((double)s_tf - Ef), w0, w1), s_j);
  const int seed_bad = hx_merge<KK>(L, true, M, rv, ri, kk, lane, wv, tid, b, 0, nullptr, nullptr);
  const double tau = seed_bad ? -INFINITY : M.tau;  // -inf: fewer than kk numeric seeds (every group qualifies)
  HX_STAMP(3);
  // the live groups into LDS, then their pairs into the queue for 2b (one
  // reservation per user: its pairs are contiguous)
  if (tid == 0) s_n = 0;
  __syncthreads();
  for (int g = tid; g < G; g += kHxThreads2) {
    if (ub_of(g) >= tau) {
      const int q = atomicAdd(&s_n, 1);
      if (q < cap2) s_glist[q] = g;
    }
  }
  __syncthreads();
  const int n_live = s_n;
  // the user's queue range (contiguous; reserved against the queue's
  // capacity); more live groups than the LDS list holds: filled window by
  // window (below), each window's odd group pairs with an empty slot, so the
  // range covers (n_live + windows) / 2 entries and the unused ones stay
  // empty pairs. No room: 2c scores every group.
  const bool big = n_live > cap2;
  const int np = big ? (n_live + (G + cap2 - 1) / cap2 + 1) / 2 : (n_live + 1) / 2;
  // (an atomicAdd, not a CAS loop: a thousand blocks retrying one CAS cost
  // 1.1 ms at B = 1024; a reservation that passes the capacity fills its
  // part below it with empty pairs, 2b reads min(total, capacity) entries)
  __shared__ int s_base, s_hole0, s_hole1;
  if (tid == 0) {
    const int cap = a.pair_capacity;
    int base = 0, h0 = 0, h1 = 0;
    if (np) {
      base = *(volatile int*)a.pair_total > cap - np ? cap : atomicAdd(a.pair_total, np);
      if (base > cap - np) h0 = base < cap ? base : cap, h1 = cap, base = -1;
    }
    s_base = base, s_hole0 = h0, s_hole1 = h1;
  }
  __syncthreads();
  const int base = s_base;
  if (base < 0) {
    for (int q = s_hole0 + tid; q < s_hole1; q += kHxThreads2) a.pairs[q] = make_int4(b, -1, -1, 0);
    if (tid == 0) {
      r.state = kHxEvery;
      r.tau = -INFINITY;
      a.rec[b] = r;
      a.counts[a.B + b] = G;
    }
    return;
  }
  if (!big) {
    for (int q = tid; q < np; q += kHxThreads2)
      a.pairs[base + q] = make_int4(b, s_glist[2 * q], 2 * q + 1 < n_live ? s_glist[2 * q + 1] : -1, 0);
  } else {
    // windows of cap2 groups: at most cap2 live ones each, paired in LDS
    // and appended to the range (the rescoring runs on every CU in 2b,
    // not on this user's one block in 2c)
    __shared__ int s_w;
    int written = 0;
    for (int g0 = 0; g0 < G; g0 += cap2) {
      const int g1 = G - g0 < cap2 ? G : g0 + cap2;
      __syncthreads();
      if (tid == 0) s_w = 0;
      __syncthreads();
      for (int g = g0 + tid; g < g1; g += kHxThreads2)
        if (ub_of(g) >= tau) s_glist[atomicAdd(&s_w, 1)] = g;
      __syncthreads();
      const int nw = s_w, pw = (nw + 1) / 2;
      for (int q = tid; q < pw; q += kHxThreads2)
        a.pairs[base + written + q] = make_int4(b, s_glist[2 * q], 2 * q + 1 < nw ? s_glist[2 * q + 1] : -1, 0);
      written += pw;
    }
    for (int q = written + tid; q < np; q += kHxThreads2) a.pairs[base + q] = make_int4(b, -1, -1, 0);
  }
  if (tid == 0) {
    r.state = kHxQueued;
    r.tau = tau;
    r.pair_base = base;
    r.n_pairs = np;
    a.rec[b] = r;
    a.counts[a.B + b] = n_live;
  }
  HX_STAMP(4);
}

#ifdef HREC_HX_STAMPS
constexpr int kHxPStampWaves = 8192;
__device__ unsigned long long g_hx_pstamps[kHxPStampWaves][4];  // start, end, pairs, exact items
#endif

// 2b. The queued pairs of every user, dealt round robin to the waves of a
// persistent grid (a user's live groups vary by an order of magnitude: a
// block per user waited on the heaviest; a pair costs about the same
// whoever's it is). Per pair: both scans, each item's fused bound against
// its user's tau, the exact two-tower chain for the items that reach it;
// the pair's best kHxSlots exact fused scores go to its own slots (no
// atomics: device-scope atomics on one counter serialised 8k pulls into
// 130 us). The user rows are read from memory (uniform loads).
template <int DK, bool FULL>
__global__ __launch_bounds__(256) void hx_pairs_kernel(HxArgs a) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int ka = FULL ? DK : a.ka, kt = FULL ? DK : a.kt;
  const int filled = *(volatile const int*)a.pair_total;  // final: 2a has completed
  const int total = filled < a.pair_capacity ? filled : a.pair_capacity;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), n_waves = gridDim.x * 4;
#ifdef HREC_HX_STAMPS
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  int n_pairs = 0, n_exact = 0;
#endif
  for (int p = gw; p < total; p += n_waves) {
    const int4 e = a.pairs[p];
    const int b = e.x;
    const HxRec r = a.rec[b];
    const HxWave<DK, FULL> W{a, a.uf + (int64_t)b * DK, a.uf + ((int64_t)a.B + b) * DK, ka, kt, lane};
    HpScale sc;
    sc.ascale = r.ascale, sc.amin_ = r.amin_, sc.tscale = r.tscale, sc.tmin_ = r.tmin_;
    int64_t j;
    const bool ok = W.item_of(e.y, e.z, j);
    float sa, tf;
    W.scan(j, ok, sa, tf);
    const bool pass = ok && hp_fuse(sc, sa, hx_up((double)tf + r.Ef), a.w0, a.w1) >= r.tau;
    const uint64_t m = __ballot(pass);
    const int n = __popcll(m);
    double* pv = a.cv + (int64_t)p * kHxSlots;
    int64_t* pi = a.ci + (int64_t)p * kHxSlots;
    if (n <= kHxSlots) {  // every passing item keeps a slot: its rank among the passing lanes
      W.exact_rounds(m, j, sa, [&](int64_t jq, float aq, float tx, int bit) {
        const int q = __popcll(m & ((1ull << bit) - 1));
        pv[q] = hp_fuse(sc, aq, tx, a.w0, a.w1);
        pi[q] = jq;
      });
    } else {  // the pair's best kHxSlots (the user's kk best are among the pairs' best kk)
      HpList<kHxSlots> L;
      L.reset();
      W.exact_rounds(m, j, sa, [&](int64_t jq, float aq, float tx, int) { L.insert(hp_fuse(sc, aq, tx, a.w0, a.w1), jq); });
      L.wave_top(kHxSlots, lane, pv, pi);
    }
    if (lane == 0) a.pc[p] = n < kHxSlots ? n : kHxSlots;
#ifdef HREC_HX_STAMPS
    ++n_pairs;
    n_exact += n;
#endif
  }
#ifdef HREC_HX_STAMPS
  if (lane == 0 && gw < kHxPStampWaves) {
    g_hx_pstamps[gw][0] = t0;
    g_hx_pstamps[gw][1] = __builtin_amdgcn_s_memtime();
    g_hx_pstamps[gw][2] = n_pairs;
    g_hx_pstamps[gw][3] = n_exact;
  }
#endif
}

// 2c. One 512-thread block per user: the stable top-k of its candidates
// (ranked in LDS), or — no bound, too many live groups or candidates, a NaN
// or a missing entry among the kk — every group of the shard scored exactly.
template <int DK, bool FULL>
__global__ __launch_bounds__(kHxThreads2) void hx_final_kernel(HxArgs a) {
#pragma clang fp contract(off)
  constexpr int KK = kHxMaxK;
  __shared__ __attribute__((aligned(16))) float sua[DK];
  __shared__ __attribute__((aligned(16))) float sut[DK];
  __shared__ double rv[8 * KK];
  __shared__ int64_t ri[8 * KK];
  __shared__ HxMergeLds M;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int b = blockIdx.x;
  const int kk = a.kk;
  const HxRec r = a.rec[b];
  if (r.state == kHxNaN) {  // NaN orders by item id: the first kk items
    if (tid < kk) {
      a.out_idx[(int64_t)b * kk + tid] = tid < a.N ? tid + a.idx_offset : -1;
      a.out_val[(int64_t)b * kk + tid] = tid < a.N ? __builtin_nan("") : 0.0;
    }
    return;
  }
  HpList<KK> L;
  L.reset();
  if (r.state == kHxQueued) {
    for (int q = r.pair_base + tid; q < r.pair_base + r.n_pairs; q += kHxThreads2) {
      const int c = a.pc[q];
      for (int e = 0; e < c; ++e) L.insert(a.cv[(int64_t)q * kHxSlots + e], a.ci[(int64_t)q * kHxSlots + e]);
    }
    if (!hx_merge<KK>(L, true, M, rv, ri, kk, lane, wv, tid, b, a.idx_offset, a.out_idx, a.out_val)) return;
  }
  // every group of the shard, exactly
  if (tid == 0) *a.flag = 1;
  const int ka = FULL ? DK : a.ka, kt = FULL ? DK : a.kt;
  for (int c = tid; c < DK; c += kHxThreads2) {
    sua[c] = a.uf[(int64_t)b * DK + c];
    sut[c] = a.uf[((int64_t)a.B + b) * DK + c];
  }
  __syncthreads();
  HpScale sc;
  sc.ascale = r.ascale, sc.amin_ = r.amin_, sc.tscale = r.tscale, sc.tmin_ = r.tmin_;
  const HxWave<DK, FULL> W{a, sua, sut, ka, kt, lane};
  L.reset();
  const int G = a.G;
  for (int p = wv; 2 * p < G; p += 8) {
    int64_t j;
    const bool ok = W.item_of(2 * p, 2 * p + 1 < G ? 2 * p + 1 : -1, j);
    float sa, tf;
    W.scan(j, ok, sa, tf);
    W.exact_rounds(__ballot(ok), j, sa,
                   [&](int64_t jq, float aq, float tx, int) { L.insert(hp_fuse(sc, aq, tx, a.w0, a.w1), jq); });
  }
  hx_merge<KK>(L, true, M, rv, ri, kk, lane, wv, tid, b, a.idx_offset, a.out_idx, a.out_val);
}

// The per-call counters: flag (modes 0 / 2: a minmax call starts the batch)
// and the pair queue's length. A kernel, not a memset: captured in a HIP
// graph, the memset node left the counters of the previous replay in place.
__global__ void hx_reset_kernel(int* flag, int n, int keep_flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && (i > 0 || !keep_flag)) flag[i] = 0;
}

struct HxWs {
  uint16_t* uop;  // [2][B][2 dk] split bf16
  float* uf;      // [2][B][dk] f32 user rows (NaN: an unknown ALS row)
  int* uok;       // [B] ALS row known
  float* stats;   // [B][G][4]
  int* counts;    // [2][B]
  int* flag;      // [0] flag, [1] pair_total
  HxRec* rec;
  int4* pairs;
  double* cv;
  int64_t* ci;
  int* pc;
  size_t total;
};

static HxWs hx_layout(char* base, int B, int64_t N, int dk) {
  HxWs w{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* r = base ? base + off : nullptr;
    off += (bytes + 255) & ~(size_t)255;
    return r;
  };
  const int64_t G = (N + kHxGrp - 1) / kHxGrp;
  w.uop = (uint16_t*)take((size_t)2 * B * dk * 4);
  w.uf = (float*)take((size_t)2 * B * dk * 4);
  w.uok = (int*)take((size_t)B * 4);
  w.stats = (float*)take((size_t)B * G * 16);
  w.counts = (int*)take((size_t)2 * B * 4);
  w.flag = (int*)take(16);  // flag, pair_total
  w.rec = (HxRec*)take((size_t)B * sizeof(HxRec));
  const size_t n_pairs = (size_t)B * hx_pair_cap((int)G);
  w.pairs = (int4*)take(n_pairs * 16);
  w.cv = (double*)take(n_pairs * kHxSlots * 8);
  w.ci = (int64_t*)take(n_pairs * kHxSlots * 8);
  w.pc = (int*)take(n_pairs * 4);
  w.total = off + 256;
  return w;
}

static size_t hx_items_bytes(int64_t N, int dk) { return (((size_t)2 * N * dk * 4 + 255) & ~(size_t)255) + 256; }
static const float* hx_norms(const void* prepared, int64_t N, int dk) {
  return reinterpret_cast<const float*>(static_cast<const char*>(prepared) + hx_items_bytes(N, dk) - 256);
}

}  // namespace hrec

using namespace hrec;

static int hx_check(const hrec_hybrid_batch* x, const char* who) {
  HREC_REQUIRE(x, "%s: null batch", who);
  HREC_REQUIRE(x->dk == 64 || x->dk == 128, "%s: dk must be 64 or 128 (got %d)", who, x->dk);
  HREC_REQUIRE(x->n_users >= 0 && x->n_users < 65536 && x->n_items >= 0 && x->n_items < 0x7fffffffll,
               "%s: bad shape", who);
  HREC_REQUIRE(x->als_width >= 1 && x->als_width <= x->dk, "%s: als_width must be in [1, dk]", who);
  HREC_REQUIRE(x->tt_width == 32 || x->tt_width == 64 || x->tt_width == 128,
               "%s: tt_width must be 32, 64 or 128 (the widths of hrec_dot_scores' f32 chain)", who);
  HREC_REQUIRE(x->tt_width <= x->dk, "%s: tt_width > dk", who);
  HREC_REQUIRE(x->als_ld >= x->als_width && x->tt_ld >= x->tt_width && x->n_als_rows >= 0,
               "%s: bad user row stride / count", who);
  HREC_REQUIRE(x->als_items_ld >= 1 && x->tt_items_ld >= x->tt_width && x->tt_items_ld % 4 == 0 &&
                   x->tt_items_t_ld >= 1,
               "%s: bad item strides (tt_items_ld: a multiple of 4 >= tt_width)", who);
  if (x->n_users == 0 || x->n_items == 0) return HREC_OK;
  HREC_REQUIRE(x->als_items_ld >= x->n_items && x->tt_items_t_ld >= x->n_items,
               "%s: transposed item strides below n_items", who);
  HREC_REQUIRE(x->als_users && x->tt_users && x->als_items_t && x->tt_items && x->tt_items_t && x->prepared,
               "%s: null pointer", who);
  HREC_REQUIRE((((uintptr_t)x->tt_items | (uintptr_t)x->prepared) & 15) == 0,
               "%s: two-tower rows / prepared operands must be 16-B aligned", who);
  return HREC_OK;
}

extern "C" size_t hrec_hybrid_exact_items_bytes(int64_t n_items, int dk) {
  return hx_items_bytes(n_items > 0 ? n_items : 0, dk);
}

extern "C" int hrec_hybrid_exact_prepare(const float* als_items_t, int64_t als_ld, int als_width,
                                         const float* tt_items, int64_t tt_ld, int tt_width, int64_t n_items, int dk,
                                         void* out, void* stream) {
  HREC_REQUIRE(dk == 64 || dk == 128, "hybrid_exact_prepare: dk must be 64 or 128");
  HREC_REQUIRE(n_items >= 0 && n_items < 0x7fffffffll, "hybrid_exact_prepare: bad n_items");
  HREC_REQUIRE(als_width >= 1 && als_width <= dk && tt_width >= 1 && tt_width <= dk,
               "hybrid_exact_prepare: widths must be in [1, dk]");
  HREC_REQUIRE(als_ld >= n_items && tt_ld >= tt_width,
               "hybrid_exact_prepare: bad strides (ALS: transposed, stride >= n_items; two-tower: row stride >= width)");
  HREC_REQUIRE(out && ((uintptr_t)out & 15) == 0, "hybrid_exact_prepare: output must be 16-B aligned");
  hipStream_t s = as_stream(stream);
  float* norms = const_cast<float*>(hx_norms(out, n_items, dk));
  if (hipMemsetAsync(norms, 0, 8, s) != hipSuccess) return check_launch("hybrid_exact_prepare: memset");
  if (n_items == 0) return HREC_OK;
  HREC_REQUIRE(als_items_t && tt_items, "hybrid_exact_prepare: null pointer");
  hipLaunchKernelGGL(hx_prepare_kernel, dim3((unsigned)((n_items + 255) / 256), 2), dim3(256), 0, s, als_items_t,
                     als_ld, als_width, tt_items, tt_ld, tt_width, n_items, dk, static_cast<uint16_t*>(out),
                     reinterpret_cast<unsigned*>(norms));
  return check_launch("hx_prepare_kernel");
}

extern "C" size_t hrec_hybrid_exact_workspace_bytes(int n_users, int64_t n_items, int dk) {
  return hx_layout(nullptr, n_users > 0 ? n_users : 0, n_items > 0 ? n_items : 0, dk).total;
}

static int hx_cus() {
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  return cus;
}

// Launches up to phase 2 (mode 0 / 2) or phase 2 alone (mode 1).
static int hx_run(const hrec_hybrid_batch* x, int mode, float* als_mm, float* tt_mm, int als_wins, int top_k,
                  int64_t idx_offset, int64_t* out_idx, double* out_val, void* workspace, hipStream_t s) {
  const int B = x->n_users, dk = x->dk;
  const int64_t N = x->n_items;
  const HxWs w = hx_layout((char*)workspace, B, N, dk);
  const int G = (int)((N + kHxGrp - 1) / kHxGrp);
  const char* items = static_cast<const char*>(x->prepared);
  {
    if (mode == 1) {  // otherwise hx_user_ops_kernel resets both
      hipLaunchKernelGGL(hx_reset_kernel, dim3(1), dim3(64), 0, s, w.flag, 2, 1);
      const int rc = check_launch("hx_reset_kernel");
      if (rc) return rc;
    }
  }
  if (mode != 1) {
    hipLaunchKernelGGL(hx_user_ops_kernel, dim3((unsigned)B, 2), dim3(128), 0, s, x->als_users, x->als_ld,
                       x->als_rows, x->n_als_rows, x->als_width, x->tt_users, x->tt_ld, x->tt_width, B, dk, w.uop,
                       w.uf, w.uok, w.flag);
    int rc = check_launch("hx_user_ops_kernel");
    if (rc) return rc;
#define HREC_HX_STATS(DK)                                                                                        \
  do {                                                                                                           \
    using S = HxShape<DK>;                                                                                       \
    const int n_ut = (B + S::UB - 1) / S::UB;                                                                    \
    /* the blocks a CU holds (the LDS holds two user tiles): item ranges of whole 32-item slices */          \
    int64_t n_rng = (S::kBlocksPerCU * hx_cus() + n_ut - 1) / n_ut;                                              \
    int64_t per = ((N + n_rng - 1) / n_rng + 31) / 32 * 32;                                                      \
    n_rng = (N + per - 1) / per;                                                                                 \
    hipLaunchKernelGGL(hx_stats_kernel<DK>, dim3((unsigned)(n_ut * n_rng)), dim3(S::kThreads), 0, s, w.uop, B,     \
                       n_ut, items, N, G, per, w.stats);                                                         \
  } while (0)
    if (dk == 64) HREC_HX_STATS(64); else HREC_HX_STATS(128);
#undef HREC_HX_STATS
    rc = check_launch("hx_stats_kernel");
    if (rc) return rc;
  }
  HxArgs a{};
  a.ka = x->als_width, a.kt = x->tt_width, a.B = B;
  a.Vat = x->als_items_t, a.lda = x->als_items_ld, a.Vt = x->tt_items, a.ldv = x->tt_items_ld;
  a.Vtt = x->tt_items_t, a.ldtt = x->tt_items_t_ld;
  a.inorm = hx_norms(x->prepared, N, dk);
  a.uf = w.uf, a.uok = w.uok;
  a.N = N, a.G = G, a.stats = w.stats;
  a.mm_a = als_mm, a.mm_t = tt_mm;
  // src/hybrid_system.py:69 — strict '>' picks (0.8, 0.2), else (0.2, 0.8)
  a.w0 = als_wins ? 0.8 : 0.2, a.w1 = als_wins ? 0.2 : 0.8;
  a.kk = (int)(top_k < N ? top_k : N);
  a.idx_offset = idx_offset, a.out_idx = out_idx, a.out_val = out_val;
  a.counts = w.counts, a.flag = w.flag;
  a.pair_cap = hx_pair_cap(G);
  a.pair_capacity = (int)((int64_t)B * a.pair_cap < 0x7fffffff ? (int64_t)B * a.pair_cap : 0x7fffffff);
  a.rec = w.rec, a.pairs = w.pairs, a.pair_total = w.flag + 1;
  a.cv = w.cv, a.ci = w.ci, a.pc = w.pc;
  const bool full = x->als_width == dk && x->tt_width == dk;
  // 2a's dynamic LDS: the user's group records (when they fit), the live groups
  const size_t st_lds = (G <= kHxStatsLds ? (size_t)G * 16 : 0) + (size_t)a.pair_cap * 8;
  // 2b: a persistent grid, 4 waves per block, four blocks per CU (<= 128 VGPRs)
  const unsigned n_pairs_blocks = (unsigned)(4 * hx_cus());
#define HREC_HX_2(DK, M, F)                                                                                      \
  do {                                                                                                           \
    if (!allow_max_lds(hx_pre_kernel<DK, M, F>)) return check_launch("hx_pre_kernel: LDS attribute");          \
    hipLaunchKernelGGL((hx_pre_kernel<DK, M, F>), dim3((unsigned)B), dim3(kHxThreads2), st_lds, s, a);          \
    int rc2 = check_launch("hx_pre_kernel");                                                                     \
    if (rc2 || M == 0) return rc2;                                                                               \
    hipLaunchKernelGGL((hx_pairs_kernel<DK, F>), dim3(n_pairs_blocks), dim3(256), 0, s, a);                    \
    rc2 = check_launch("hx_pairs_kernel");                                                                       \
    if (rc2) return rc2;                                                                                         \
    hipLaunchKernelGGL((hx_final_kernel<DK, F>), dim3((unsigned)B), dim3(kHxThreads2), 0, s, a);                \
    return check_launch("hx_final_kernel");                                                                      \
  } while (0)
#define HREC_HX_M(DK, M)                 \
  do {                                   \
    if (full) HREC_HX_2(DK, M, true);    \
    else HREC_HX_2(DK, M, false);        \
  } while (0)
  if (dk == 64) {
    if (mode == 0) HREC_HX_M(64, 0); else if (mode == 1) HREC_HX_M(64, 1); else HREC_HX_M(64, 2);
  } else {
    if (mode == 0) HREC_HX_M(128, 0); else if (mode == 1) HREC_HX_M(128, 1); else HREC_HX_M(128, 2);
  }
#undef HREC_HX_M
#undef HREC_HX_2
}

extern "C" int hrec_hybrid_exact_minmax(const hrec_hybrid_batch* x, float* als_mm, float* tt_mm, void* workspace,
                                        size_t workspace_bytes, void* stream) {
  int rc = hx_check(x, "hybrid_exact_minmax");
  if (rc) return rc;
  if (x->n_users == 0) return HREC_OK;
  HREC_REQUIRE(als_mm && tt_mm && workspace, "hybrid_exact_minmax: null output or workspace");
  hipStream_t s = as_stream(stream);
  if (x->n_items == 0) {  // no items: min = +inf, max = -inf (hrec_rows_minmax_f32 of an empty row)
    const float inf = INFINITY;
    float h[2] = {inf, -inf};
    for (int m = 0; m < 2; ++m)
      for (int q = 0; q < 2; ++q)
        if (hipMemsetD32Async((hipDeviceptr_t)((m ? tt_mm : als_mm) + (size_t)q * x->n_users),
                              *reinterpret_cast<int*>(&h[q]), x->n_users, s) != hipSuccess)
          return check_launch("hybrid_exact_minmax: memset");
    return HREC_OK;
  }
  const size_t need = hrec_hybrid_exact_workspace_bytes(x->n_users, x->n_items, x->dk);
  HREC_REQUIRE(workspace_bytes >= need, "hybrid_exact_minmax: workspace %zu < %zu", workspace_bytes, need);
  return hx_run(x, 0, als_mm, tt_mm, 0, 1, 0, nullptr, nullptr, workspace, s);
}

extern "C" int hrec_hybrid_exact_topk(const hrec_hybrid_batch* x, const float* als_mm, const float* tt_mm,
                                      int als_wins, int top_k, int64_t idx_offset, int64_t* out_idx, double* out_val,
                                      void* workspace, size_t workspace_bytes, void* stream) {
  int rc = hx_check(x, "hybrid_exact_topk");
  if (rc) return rc;
  HREC_REQUIRE(top_k >= 1 && top_k <= kHxMaxK, "hybrid_exact_topk: top_k must be in [1, %d] (larger: the unfused path)",
               kHxMaxK);
  if (x->n_users == 0 || x->n_items == 0) return HREC_OK;
  HREC_REQUIRE(als_mm && tt_mm && out_idx && out_val && workspace, "hybrid_exact_topk: null pointer");
  const size_t need = hrec_hybrid_exact_workspace_bytes(x->n_users, x->n_items, x->dk);
  HREC_REQUIRE(workspace_bytes >= need, "hybrid_exact_topk: workspace %zu < %zu", workspace_bytes, need);
  return hx_run(x, 1, const_cast<float*>(als_mm), const_cast<float*>(tt_mm), als_wins, top_k, idx_offset, out_idx,
                out_val, workspace, as_stream(stream));
}

extern "C" int hrec_hybrid_exact_local(const hrec_hybrid_batch* x, int als_wins, int top_k, int64_t idx_offset,
                                       float* als_mm, float* tt_mm, int64_t* out_idx, double* out_val,
                                       void* workspace, size_t workspace_bytes, void* stream) {
  int rc = hx_check(x, "hybrid_exact_local");
  if (rc) return rc;
  HREC_REQUIRE(top_k >= 1 && top_k <= kHxMaxK, "hybrid_exact_local: top_k must be in [1, %d] (larger: the unfused path)",
               kHxMaxK);
  if (x->n_users == 0) return HREC_OK;
  if (x->n_items == 0)  // extremes of an empty shard; no top-k entries
    return hrec_hybrid_exact_minmax(x, als_mm, tt_mm, workspace, workspace_bytes, stream);
  HREC_REQUIRE(als_mm && tt_mm && out_idx && out_val && workspace, "hybrid_exact_local: null pointer");
  const size_t need = hrec_hybrid_exact_workspace_bytes(x->n_users, x->n_items, x->dk);
  HREC_REQUIRE(workspace_bytes >= need, "hybrid_exact_local: workspace %zu < %zu", workspace_bytes, need);
  return hx_run(x, 2, als_mm, tt_mm, als_wins, top_k, idx_offset, out_idx, out_val, workspace, as_stream(stream));
}

extern "C" int hrec_hybrid_exact_counts(const void* workspace, int n_users, int64_t n_items, int dk, int32_t* out,
                                        void* stream) {
  HREC_REQUIRE(workspace && out && n_users >= 0 && n_items >= 0 && (dk == 64 || dk == 128),
               "hybrid_exact_counts: bad argument");
  const HxWs w = hx_layout((char*)workspace, n_users, n_items, dk);
  hipStream_t s = as_stream(stream);
  if (n_users > 0 && hipMemcpyAsync(out, w.counts, (size_t)2 * n_users * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return check_launch("hybrid_exact_counts: copy");
  if (hipMemcpyAsync(out + 2 * (size_t)n_users, w.flag, 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return check_launch("hybrid_exact_counts: copy");
  return HREC_OK;
}

#ifdef HREC_HX_STAMPS
extern "C" int hrec_debug_hx1_stamps(unsigned long long* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_hx1_stamps), sizeof(g_hx1_stamps)) == hipSuccess ? 0 : -2;
}
extern "C" int hrec_debug_hx_pstamps(unsigned long long* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_hx_pstamps), sizeof(g_hx_pstamps)) == hipSuccess ? 0 : -2;
}
extern "C" int hrec_debug_hx_stamps(unsigned long long* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_hx_stamps), sizeof(g_hx_stamps)) == hipSuccess ? 0 : -2;
}
#endif
