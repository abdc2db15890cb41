// K9p: the bf16 hybrid top-k of BASELINE config c5 without writing either
// [B, N] score matrix — what get_hybrid_recommendations does per user
// (src/hybrid_system.py:95-116: ALS transform + Keras Dot over every
// candidate, one MinMaxScaler per model, 0.8 / 0.2 fusion, stable
// sorted()[:top_k]) for a batch of users over an item shard.
//
// The fusion needs each user's min / max of BOTH score rows before any fused
// score exists, so the scores are computed twice, the second time for one
// model only:
//   phase 1 (hrec_hybrid_prune_minmax): the user rows gathered + converted to
//     bf16 operands once; both GEMMs (hyb_scores_kernel, mode HS_PRUNE: no
//     stores) -> per-user min / max of both rows, and per item group (block)
//     both models' group maxima + the 16-NI item slice holding the heavy one;
//   [the caller all-reduces the min / max across item shards (C2)]
//   phase 2 (hrec_hybrid_prune_topk), three launches:
//     a. bound: per user, the slices of the 16 groups with the largest maxima
//        of the HEAVY model (weight 0.8); both scores of these seeds by the
//        exact path's MFMA chains -> exact fused scores, tau = their k-th
//        best <= the shard's k-th best. An item of group g in the top k has
//        w_h h_n >= tau - w_l l_n with l_n <= the light model's group maximum
//        scaled, hence a raw heavy score >= theta_g (f64, lowered by a
//        relative margin); +inf where the group's heavy maximum is below it;
//     b. the heavy model's GEMM alone with the per-group survivor filter
//        (hyb_scores_kernel HS_FILTER: one block per item group, so a user's
//        bound is one LDS value per block; survivors staged in LDS and
//        flushed once per block): item ids + exact heavy scores per user;
//     c. each survivor's light score with the same bf16 MFMA k order (A =
//        the gathered item rows, B = the user row), the fused score with
//        fuse_rows_kernel's arithmetic (ALS branch f64, two-tower f32, numpy
//        1.21 promotion), the exact stable top-k (ties -> smaller item) —
//        and, in the same block, the exact path over every item of the shard
//        for a user without a bound (non-finite extremes), with an
//        overflowing or short list, or with a NaN among its k: no fallback
//        launch and no host round trip, so a batch can be captured as one
//        HIP graph.
// Bit-identical to hrec_hybrid_scores + hrec_fuse_rows_topk: every score is
// the same MFMA chain and every fused score the same arithmetic.
#include <float.h>
#include <math.h>

#include "common.h"
#include "hybrid_common.h"

namespace hrec {

typedef __bf16 hp_bf8 __attribute__((ext_vector_type(8)));

union HpFrag {
  int4 i;
  hp_f4 f;
};

constexpr int kHpCap = 8192;      // survivors per user (expected: a few hundred)
static_assert(kHpCap >= 256, "hp_cand_topk_kernel reads the first 256 slots unconditionally");
constexpr int kHpMaxK = 8;        // top_k handled here (kFuseK of the exact path)
constexpr int kHpMaxGroups = 16;  // heavy-model groups whose max slices seed the bound

__device__ __forceinline__ float hp_f(uint32_t bits16) { return __uint_as_float(bits16 << 16); }

#ifdef HREC_HP_STAMPS
// Diagnostic builds only: per block (thread 0) s_memtime at the kernel's
// phase points, [kernel 0 = bound, 1 = survivors][block][point], plain stores.
constexpr int kHpStampBlocks = 1024;
__device__ unsigned long long g_hp_stamps[2][kHpStampBlocks][8];
#define HP_STAMP_DECL unsigned long long hp_t[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define HP_STAMP(i)                                          \
  do {                                                       \
    if (threadIdx.x == 0) hp_t[i] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define HP_STAMP_OUT(kid)                                                            \
  do {                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < kHpStampBlocks) {                           \
      hp_t[7] = __builtin_amdgcn_s_memtime();                                        \
      for (int _q = 0; _q < 8; ++_q) g_hp_stamps[kid][blockIdx.x][_q] = hp_t[_q];    \
    }                                                                                \
  } while (0)
#else
#define HP_STAMP_DECL
#define HP_STAMP(i)
#define HP_STAMP_OUT(kid)
#endif

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 1. bf16 user operands [2][B][dk]: the ALS rows gathered by als_rows (a row
// outside [0, n_als_rows) reads as NaN, as hyb_scores_kernel stages it) and
// the two-tower rows, columns >= width zero — hyb_scores_kernel's staging.
// (Folding this into phase 1 — every GEMM block gathering and converting its
// f32 rows — measured slower: phase 1 35.7 -> 47.7 us against this launch's
// 5.4 us, round 4.)
__global__ __launch_bounds__(256) void hp_user_ops_kernel(const float* __restrict__ als_users, int64_t als_ld,
                                                          const int64_t* __restrict__ als_rows, int64_t n_als_rows,
                                                          int als_width, const float* __restrict__ tt_users,
                                                          int64_t tt_ld, int tt_width, int B, int dk,
                                                          uint16_t* __restrict__ uop) {
  const int b = blockIdx.x, m = blockIdx.y;
  const float* src = m ? tt_users : als_users;
  const int64_t ld = m ? tt_ld : als_ld;
  const int wd = m ? tt_width : als_width;
  int64_t row = b;
  bool bad = false;
  if (m == 0 && als_rows) {
    row = als_rows[b];
    bad = row < 0 || row >= n_als_rows;
  }
  uint16_t* out = uop + ((int64_t)m * B + b) * dk;
  for (int c = threadIdx.x; c < dk; c += blockDim.x) {
    float v = 0.f;
    if (c < wd) v = bad ? __builtin_nanf("") : src[row * ld + c];
    out[c] = (uint16_t)hp_bf16(v);
  }
}

// 16 gathered item rows (A, row c = item c) against one user row (B, every
// column the same user): acc[r] of lane (g, c) = the score of item 4 g + r,
// the k order of hyb_scores_kernel / dot_res_kernel (bit-identical scores).
// A padding slot (item < 0) reads row 0; its result is dropped.
template <int DK>
__device__ __forceinline__ void hp_gather_load(const char* __restrict__ vbase, int64_t item, int64_t N, int g,
                                               HpFrag (&it)[DK / 32]) {
  constexpr int KS = DK / 32;
  // survivors are arbitrary rows: 64-bit addresses (a buffer resource spans at most 4 GiB)
  const char* row = vbase + (item >= 0 && item < N ? item : 0) * (int64_t)(DK * 2);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) it[ks].i = *reinterpret_cast<const int4*>(row + 16 * g + 64 * ks);
}

template <int DK>
__device__ __forceinline__ hp_f4 hp_dot(const HpFrag (&it)[DK / 32], const HpFrag (&uf)[DK / 32]) {
  hp_f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < DK / 32; ++ks)
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(hp_bf8, it[ks].i),
                                                  __builtin_bit_cast(hp_bf8, uf[ks].i), acc, 0, 0, 0);
  return acc;
}

// Order point between a batch of row loads and the MFMAs that use them: left
// to itself the scheduler interleaves each load with the MFMA of the one
// before (a few loads in flight, one round trip per k-step); with every load
// of the batch issued first, the batch costs one round trip.
__device__ __forceinline__ void hp_loads_issued() { __builtin_amdgcn_sched_barrier(0); }

// 2a. The bound: one 256-thread block per user. Seeds = the item slices of
// the kHpMaxGroups groups with the largest heavy-model maxima (4 NI items
// each); both scores of every seed by the same MFMA chain as the exact path,
// so their fused scores are exact and tau = the kk-th best of them is a lower
// bound of the shard's kk-th best. Then per item group gi a bound on the heavy
// raw score: an item of gi in the top kk has w_h h_n >= tau - w_l l_n and l_n
// <= the light model's group maximum scaled (pass 1's partials), so theta_gi
// = the raw score of that h_n, lowered by a relative margin. Also resets the
// user's survivor count, and block 0 the fallback flag.
// LOCAL (hrec_hybrid_prune_local, one shard): the user's row extremes are
// first reduced here from phase 1's group partials (and written out), in
// place of hyb_mm_reduce_kernel + a separate bound launch.
template <int DK, bool LOCAL>
__global__ __launch_bounds__(256) void hp_bound_kernel(const float* __restrict__ part, const int* __restrict__ argpos,
                                                       int G, int64_t N, int B, int hm, const float* __restrict__ als_mm,
                                                       const float* __restrict__ tt_mm, float* __restrict__ als_mm_out,
                                                       float* __restrict__ tt_mm_out, double w0, double w1, int kk,
                                                       int slice_ni, const uint16_t* __restrict__ uop,
                                                       const uint16_t* __restrict__ als_items,
                                                       const uint16_t* __restrict__ tt_items,
                                                       float* __restrict__ theta, int* __restrict__ cn,
                                                       int* __restrict__ uflag, int* __restrict__ flag) {
#pragma clang fp contract(off)
  constexpr int KS = DK / 32;
  constexpr int kSlots = kHpMaxGroups * 16;  // <= 16 groups x (4 NI <= 16) items
  __shared__ __attribute__((aligned(16))) float smax[128];
  __shared__ int srank[128];
  __shared__ int sitem[kSlots];
  __shared__ __attribute__((aligned(16))) double sfl[kSlots];
  __shared__ double s_tau;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  HP_STAMP_DECL;
  HP_STAMP(0);
  const int b = blockIdx.x;
  if (b == 0 && tid == 0) *flag = 0;
  if (tid == 0) cn[b] = 0;
  float* th_row = theta + (int64_t)b * G;
  // every load the bound needs besides the seeds' rows, issued before the
  // extremes are known (one round trip): the user's bf16 rows (B operands of
  // the seed MFMAs), the heavy group maxima (+ their slices), the light ones
  const char* uh = reinterpret_cast<const char*>(uop + ((int64_t)hm * B + b) * DK);
  const char* ul = reinterpret_cast<const char*>(uop + ((int64_t)(1 - hm) * B + b) * DK);
  HpFrag fh[KS], fl[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    fh[ks].i = *reinterpret_cast<const int4*>(uh + 16 * g + 64 * ks);
    fl[ks].i = *reinterpret_cast<const int4*>(ul + 16 * g + 64 * ks);
  }
  const int lm = 1 - hm;
  float lmx = -INFINITY;
  int ap = -1;  // the group's max slice (kept for the seed slots below: no second load)
  if (tid < 128) {
    float v = -INFINITY;
    if (tid < G) {
      ap = argpos[((int64_t)hm * G + tid) * B + b];
      const float pv = part[(((int64_t)hm * G + tid) * 2 + 1) * B + b];
      lmx = part[(((int64_t)lm * G + tid) * 2 + 1) * B + b];
      v = ap >= 0 ? pv : -INFINITY;
    }
    smax[tid] = v;
  }
  float amin, amax, tmin, tmax;
  if constexpr (LOCAL) {
    // thread t: model t >> 7, group t & 127 (G <= 128); fminf / fmaxf as
    // hyb_mm_reduce_kernel (exact: the same extremes)
    __shared__ float red[4][2];
    const int m = tid >> 7, gi = tid & 127;
    float lo = INFINITY, hi = -INFINITY;
    if (gi < G) {
      lo = part[(((int64_t)m * G + gi) * 2) * B + b];
      hi = part[(((int64_t)m * G + gi) * 2 + 1) * B + b];
    }
    // wave min / max without LDS permutes: DPP within rows (quad swaps, half-
    // row and row mirrors), then the row / half swaps of gfx950
    lo = fminf(lo, hp_dpp32<0xB1>(lo));
    hi = fmaxf(hi, hp_dpp32<0xB1>(hi));
    lo = fminf(lo, hp_dpp32<0x4E>(lo));
    hi = fmaxf(hi, hp_dpp32<0x4E>(hi));
    lo = fminf(lo, hp_dpp32<0x141>(lo));
    hi = fmaxf(hi, hp_dpp32<0x141>(hi));
    lo = fminf(lo, hp_dpp32<0x140>(lo));
    hi = fmaxf(hi, hp_dpp32<0x140>(hi));
    lo = fminf(lo, hp_xor16(lo));
    hi = fmaxf(hi, hp_xor16(hi));
    lo = fminf(lo, hp_xor32(lo));
    hi = fmaxf(hi, hp_xor32(hi));
    if (lane == 0) {
      red[wv][0] = lo;
      red[wv][1] = hi;
    }
    __syncthreads();
    HP_STAMP(1);
    amin = fminf(red[0][0], red[1][0]);
    amax = fmaxf(red[0][1], red[1][1]);
    tmin = fminf(red[2][0], red[3][0]);
    tmax = fmaxf(red[2][1], red[3][1]);
    if (tid == 0) {
      als_mm_out[b] = amin;
      als_mm_out[B + b] = amax;
      tt_mm_out[b] = tmin;
      tt_mm_out[B + b] = tmax;
    }
  } else {
    amin = als_mm[b], amax = als_mm[B + b], tmin = tt_mm[b], tmax = tt_mm[B + b];
  }
  if (!(isfinite(amin) && isfinite(amax) && isfinite(tmin) && isfinite(tmax))) {
    // NaN / infinite scores (an unknown user row, non-finite vectors): the
    // exact path ranks them; nothing survives the filter
    for (int gi = tid; gi < G; gi += 256) th_row[gi] = INFINITY;
    if (tid == 0) uflag[b] = 1;
    HP_STAMP_OUT(0);
    return;  // block-uniform
  }
  const HpScale sc = hp_scale(amin, amax, tmin, tmax);
  const int64_t per = ((N + G - 1) / G + 15) / 16 * 16;  // hyb_scores_kernel's group range
  for (int q = tid; q < kSlots; q += 256) sitem[q] = -1;
  if (tid == 0) s_tau = -INFINITY;
  __syncthreads();
  HP_STAMP(2);
  // the kHpMaxGroups largest group maxima (value desc, group asc) -> seed
  // slots. Group gi's rank over all 128 slots (those >= G hold -inf, never
  // counted) in two halves: thread gi the lower, thread 128 + gi the upper,
  // 16 broadcast 16-B reads each; non-short-circuit forms (a branch per
  // element would wait for each read)
  const int per_g = 4 * slice_ni;
  {
    const int gi = tid & 127, h = tid >> 7;
    const float v = smax[gi];
    int part_rank = 0;
#pragma unroll
    for (int q0 = 0; q0 < 64; q0 += 4) {
      const int q = 64 * h + q0;
      const float4 o = *reinterpret_cast<const float4*>(smax + q);
      part_rank += (int)(o.x > v) | ((int)(o.x == v) & (int)(q < gi));
      part_rank += (int)(o.y > v) | ((int)(o.y == v) & (int)(q + 1 < gi));
      part_rank += (int)(o.z > v) | ((int)(o.z == v) & (int)(q + 2 < gi));
      part_rank += (int)(o.w > v) | ((int)(o.w == v) & (int)(q + 3 < gi));
    }
    if (h == 1) srank[gi] = part_rank;
    __syncthreads();
    if (h == 0 && gi < G && v != -INFINITY) {
      const int rank = part_rank + srank[gi];
      if (rank < kHpMaxGroups) {
        const int pos = ap;
        const int64_t jb = (int64_t)(pos >> 2) * 16;
        const int gq = pos & 3;
        const int64_t i1 = (int64_t)tid * per + per < N ? (int64_t)tid * per + per : N;
        for (int t = 0; t < slice_ni; ++t)
          for (int r = 0; r < 4; ++r) {
            const int64_t j = jb + 16 * t + 4 * gq + r;
            sitem[rank * per_g + 4 * t + r] = j < i1 ? (int)j : -1;
          }
      }
    }
  }
  __syncthreads();
  HP_STAMP(3);
  // exact fused scores of the seeds: 16 per MFMA group, both models; the 4
  // waves take groups (w, w + 4), then (w + 8, w + 12) when the slices hold 4
  // tiles, all rows of a pair in flight at once
  const char* vh = reinterpret_cast<const char*>(hm ? tt_items : als_items);
  const char* vl = reinterpret_cast<const char*>(hm ? als_items : tt_items);
  const int n_slots = kHpMaxGroups * per_g;
  auto seed = [&](int q, const hp_f4& ah, const hp_f4& al, int item) {
    const int slot = 16 * q + 4 * g + (c & 3);
    const int it_s = __shfl(item, 4 * g + (c & 3), kWave);
    if (c < 4) {
      const float h = hp_pick(ah, c), l = hp_pick(al, c);
      const double f = hm ? hp_fuse(sc, l, h, w0, w1) : hp_fuse(sc, h, l, w0, w1);
      sfl[slot] = (it_s >= 0 && f == f) ? f : -INFINITY;
    }
  };
  for (int q = wv; 16 * q < n_slots; q += 8) {
    const int q2 = q + 4;
    const int item = sitem[16 * q + c];
    const int item2 = 16 * q2 < n_slots ? sitem[16 * q2 + c] : -1;
    HpFrag rh[KS], rl[KS];
    hp_gather_load<DK>(vh, item, N, g, rh);
    hp_gather_load<DK>(vl, item, N, g, rl);
    if (16 * q2 < n_slots) {  // wave-uniform
      HpFrag rh2[KS], rl2[KS];
      hp_gather_load<DK>(vh, item2, N, g, rh2);
      hp_gather_load<DK>(vl, item2, N, g, rl2);
      hp_loads_issued();
      seed(q, hp_dot<DK>(rh, fh), hp_dot<DK>(rl, fl), item);
      seed(q2, hp_dot<DK>(rh2, fh), hp_dot<DK>(rl2, fl), item2);
    } else {
      hp_loads_issued();
      seed(q, hp_dot<DK>(rh, fh), hp_dot<DK>(rl, fl), item);
    }
  }
  __syncthreads();
  HP_STAMP(4);
  // tau = the kk-th largest (the seed items are distinct): the thread pair
  // (2 q, 2 q + 1) ranks slot q over the two halves of the list
  const int half = n_slots / 2;  // a multiple of 16
  for (int qq = tid; qq < 2 * n_slots; qq += 256) {
    const int q = qq >> 1, h = qq & 1;
    const double v = sfl[q];
    int rank = 0;
    if (v != -INFINITY) {
      for (int o0 = h * half; o0 < (h + 1) * half; o0 += 16) {  // 8 broadcast 16-B reads in flight
#pragma unroll
        for (int e = 0; e < 16; e += 2) {
          const double2 x = *reinterpret_cast<const double2*>(sfl + o0 + e);
          rank += (int)(x.x > v) | ((int)(x.x == v) & (int)(o0 + e < q));
          rank += (int)(x.y > v) | ((int)(x.y == v) & (int)(o0 + e + 1 < q));
        }
      }
    }
    rank += __shfl_xor(rank, 1, kWave);
    if (h == 0 && v != -INFINITY && rank == kk - 1) s_tau = v;
  }
  __syncthreads();
  HP_STAMP(5);
  const double tau = s_tau;
  if (tau == -INFINITY) {  // fewer than kk numeric seeds: the exact path
    for (int gi = tid; gi < G; gi += 256) th_row[gi] = INFINITY;
    if (tid == 0) uflag[b] = 1;
    HP_STAMP_OUT(0);
    return;
  }
  if (tid == 0) uflag[b] = 0;
  for (int gi = tid; gi < G; gi += 256) {  // G <= 128: gi == tid, lmx loaded above
    float th = INFINITY;  // no numeric light score in the group: fused NaN, below the kk seeds
    if (lmx > -INFINITY) {
      if (hm == 0) {  // heavy = ALS (w0): a_n >= (tau - w1 t_n) / w0, t_n <= the group's max scaled
        const float tn_max = lmx * sc.tscale + sc.tmin_;
        const double hn = (tau - w1 * (double)tn_max) / w0 - 1e-9;
        double x = (hn - sc.amin_) / sc.ascale;
        x -= 1e-6 * (fabs(x) + ((double)amax - (double)amin));
        th = (float)x;
        if ((double)th > x) th = nextafterf(th, -INFINITY);
      } else {  // heavy = two-tower (w1): t_n >= (tau - w0 a_n) / w1
        const double an_max = (double)lmx * sc.ascale + sc.amin_;
        const double hn = (tau - w0 * an_max) / w1 - 1e-9;
        double x = (hn - (double)sc.tmin_) / (double)sc.tscale;
        x -= 1e-6 * (fabs(x) + ((double)tmax - (double)tmin));
        th = (float)x;
        if ((double)th > x) th = nextafterf(th, -INFINITY);
      }
    }
    // the group's heavy maximum is below its bound: nothing of it survives
    // (+inf: the filter skips the group's tiles for this user)
    if (gi < 128 && (double)th > (double)smax[gi]) th = INFINITY;
    th_row[gi] = th;
  }
  HP_STAMP_OUT(0);
}

// 2c. Survivors of user blockIdx.x (8 waves, 16 survivors per MFMA group):
// light scores, fused scores, each lane's sorted best kk, each wave's best
// kk, wave 0 merges -> the user's top kk (+ idx_offset). A flagged user (no
// bound, non-finite extremes), an overflowing / short list, or a NaN among the
// kk (the exact order then depends on the NaN items of the whole shard) takes
// the exact path IN THE SAME BLOCK: both scores of every item of the shard
// by the same MFMA chains, the same fusion and the same order — so no
// fallback launch exists, and only the users that need it pay for it. (All
// of one model's scores NaN, e.g. an unknown user: every fused score is NaN
// and the top kk are the shard's first kk items.) Sets *flag when any user
// took the exact path.
template <int DK>
__global__ __launch_bounds__(512) void hp_cand_topk_kernel(const int* __restrict__ cn, int cap,
                                                           const float* __restrict__ cv, const int64_t* __restrict__ ci,
                                                           const int* __restrict__ uflag,
                                                           const uint16_t* __restrict__ uop, int hm,
                                                           const void* __restrict__ als_items,
                                                           const void* __restrict__ tt_items, int64_t N, int B,
                                                           const float* __restrict__ als_mm,
                                                           const float* __restrict__ tt_mm, double w0, double w1,
                                                           int kk, int64_t idx_offset, int64_t* __restrict__ out_idx,
                                                           double* __restrict__ out_val, int* __restrict__ flag) {
  constexpr int KS = DK / 32, KK = kHpMaxK;
  __shared__ double rv[8 * KK];
  __shared__ int64_t ri[8 * KK];
  __shared__ int s_full;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  HP_STAMP_DECL;
  HP_STAMP(0);
  const int b = blockIdx.x;
  const float* cvb = cv + (int64_t)b * cap;
  const int64_t* cib = ci + (int64_t)b * cap;
  const char* vh = static_cast<const char*>(hm ? tt_items : als_items);
  const char* vl = static_cast<const char*>(hm ? als_items : tt_items);
  // the wave's first two survivor groups (ids of rows c, heavy scores of
  // slots 4 g + (c & 3)) load with the count: slots < cap always exist
  const int hs = 4 * g + (c & 3);
  int q0 = wv;
  int64_t n_it0 = cib[16 * q0 + c], n_it1 = cib[16 * (q0 + 8) + c];
  float n_h0 = cvb[16 * q0 + hs], n_h1 = cvb[16 * (q0 + 8) + hs];
  const char* ur = reinterpret_cast<const char*>(uop + ((int64_t)(1 - hm) * B + b) * DK);
  HpFrag uf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) uf[ks].i = *reinterpret_cast<const int4*>(ur + 16 * g + 64 * ks);
  const int nb = cn[b];
  const bool flagged = uflag[b] || nb > cap || nb < kk;  // block-uniform
  const float amin = als_mm[b], amax = als_mm[B + b], tmin = tt_mm[b], tmax = tt_mm[B + b];
  const HpScale sc = hp_scale(amin, amax, tmin, tmax);
  double lv[KK];
  int64_t li[KK];
  auto reset = [&]() {
#pragma unroll
    for (int j = 0; j < KK; ++j) {
      lv[j] = 0.0;
      li[j] = INT64_MAX;  // empty slot
    }
  };
  auto insert = [&](double xv, int64_t xi) {
#pragma unroll
    for (int j = 0; j < KK; ++j) {  // compare-exchange chain (sorted list)
      const bool sw = li[j] == INT64_MAX || hp_better(xv, xi, lv[j], li[j]);
      const double tv = lv[j];
      const int64_t ti = li[j];
      lv[j] = sw ? xv : tv;
      li[j] = sw ? xi : ti;
      xv = sw ? tv : xv;
      xi = sw ? ti : xi;
    }
  };
  auto fused = [&](float h, float l) { return hm ? hp_fuse(sc, l, h, w0, w1) : hp_fuse(sc, h, l, w0, w1); };
  auto wave_best = [&](double& bv, int64_t& bi) { hp_wave_best(bv, bi); };  // csrc/hybrid_common.h
  // the lanes' lists -> each wave's best kk (LDS) -> wave 0's merge; writes
  // the outputs when `write`; returns (in s_full) whether a NaN or a missing
  // entry is among the kk. Called block-uniformly.
  auto merge = [&](bool write) {
    for (int r = 0; r < kk; ++r) {
      double bv = lv[0];
      int64_t bi = li[0];
      wave_best(bv, bi);
      if (lane == 0) {
        rv[wv * KK + r] = bv;
        ri[wv * KK + r] = bi;
      }
      if (bi != INT64_MAX && li[0] == bi) {  // the (unique) owner pops its head
#pragma unroll
        for (int j = 0; j + 1 < KK; ++j) {
          lv[j] = lv[j + 1];
          li[j] = li[j + 1];
        }
        li[KK - 1] = INT64_MAX;
      }
    }
    __syncthreads();
    if (wv == 0) {
      // lane l holds candidates l (and l + 64 when 8 kk > 64), better one first
      double v0 = 0.0, v1 = 0.0;
      int64_t i0 = INT64_MAX, i1 = INT64_MAX;
      if (lane < 8 * KK && (lane % KK) < kk) {
        v0 = rv[lane];
        i0 = ri[lane];
      }
      if (lane + 64 < 8 * KK && ((lane + 64) % KK) < kk) {
        v1 = rv[lane + 64];
        i1 = ri[lane + 64];
      }
      if (i1 != INT64_MAX && (i0 == INT64_MAX || hp_better(v1, i1, v0, i0))) {
        const double tv = v0;
        const int64_t ti = i0;
        v0 = v1;
        i0 = i1;
        v1 = tv;
        i1 = ti;
      }
      bool bad = false;
      for (int r = 0; r < kk; ++r) {
        double bv = v0;
        int64_t bi = i0;
        wave_best(bv, bi);
        if (bi == INT64_MAX || bv != bv) bad = true;
        if (write && lane == 0) {
          out_idx[(int64_t)b * kk + r] = bi == INT64_MAX ? -1 : bi + idx_offset;
          out_val[(int64_t)b * kk + r] = bi == INT64_MAX ? 0.0 : bv;
        }
        if (bi != INT64_MAX && i0 == bi) {
          v0 = v1;
          i0 = i1;
          i1 = INT64_MAX;
        }
      }
      if (lane == 0) s_full = bad ? 1 : 0;
    }
    __syncthreads();
  };
  HP_STAMP(1);
  reset();
  if (!flagged) {
    // two survivor groups per wave in flight (q0, q0 + 8); the next pair's
    // ids and heavy scores load while this pair's rows are gathered
    auto take = [&](const hp_f4& acc, int q, int64_t item, float h) {
      const int p = 16 * q + hs;
      const int64_t pid = __shfl(item, hs, kWave);
      if (c < 4 && p < nb) insert(fused(h, hp_pick(acc, c)), pid);
    };
    for (; 16 * q0 < nb; q0 += 16) {
      const int q1 = q0 + 8;
      const int64_t it0 = 16 * q0 + c < nb ? n_it0 : -1;
      const int64_t it1 = 16 * q1 + c < nb ? n_it1 : -1;
      const float h0 = n_h0, h1 = n_h1;
      const int qn = q0 + 16;
      if (16 * qn < nb) {
        n_it0 = cib[16 * qn + c];
        n_h0 = cvb[16 * qn + hs];
        if (16 * (qn + 8) < cap) {
          n_it1 = cib[16 * (qn + 8) + c];
          n_h1 = cvb[16 * (qn + 8) + hs];
        }
      }
      HpFrag r0[KS];
      hp_gather_load<DK>(vl, it0, N, g, r0);
      if (16 * q1 < nb) {  // wave-uniform
        HpFrag r1[KS];
        hp_gather_load<DK>(vl, it1, N, g, r1);
        hp_loads_issued();
        take(hp_dot<DK>(r0, uf), q0, it0, h0);
        take(hp_dot<DK>(r1, uf), q1, it1, h1);
      } else {
        hp_loads_issued();
        take(hp_dot<DK>(r0, uf), q0, it0, h0);
      }
    }
  }
  HP_STAMP(2);
  merge(!flagged);
  const bool done = !flagged && s_full == 0;
  HP_STAMP(3);
  if (done) {  // block-uniform
    HP_STAMP_OUT(1);
    return;
  }
  // the exact path for this user
  if (tid == 0) *flag = 1;
  if (!(amin <= amax) || !(tmin <= tmax)) {
    // one model has no number at all: every fused score is NaN, and NaN
    // orders by item id
    if (tid < kk) {
      out_idx[(int64_t)b * kk + tid] = tid < N ? tid + idx_offset : -1;
      out_val[(int64_t)b * kk + tid] = tid < N ? __builtin_nan("") : 0.0;
    }
    return;
  }
  const char* uhr = reinterpret_cast<const char*>(uop + ((int64_t)hm * B + b) * DK);
  HpFrag uh[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) uh[ks].i = *reinterpret_cast<const int4*>(uhr + 16 * g + 64 * ks);
  reset();
  for (int64_t q = wv; 16 * q < N; q += 8) {
    const int64_t item = 16 * q + c < N ? 16 * q + c : -1;
    HpFrag rh[KS], rl[KS];
    hp_gather_load<DK>(vh, item, N, g, rh);
    hp_gather_load<DK>(vl, item, N, g, rl);
    hp_loads_issued();
    const hp_f4 ah = hp_dot<DK>(rh, uh);
    const hp_f4 al = hp_dot<DK>(rl, uf);
    const int64_t p = 16 * q + hs;
    if (c < 4 && p < N) insert(fused(hp_pick(ah, c), hp_pick(al, c)), p);
  }
  merge(true);
}

struct HpWs {
  float* part;
  int* argpos;
  uint16_t* uop;
  float* theta;  // [B][G] heavy raw-score bound per item group
  int* uflag;    // [B] the bound's per-user fallback reason
  float* cv;
  int64_t* ci;
  int* cn;
  int* flag;
  size_t total;
};

static HpWs hp_layout(char* base, int B, int64_t N, int dk, int kk) {
  HpWs w{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* r = base ? base + off : nullptr;
    off += (bytes + 255) & ~(size_t)255;
    return r;
  };
  const int G = hs_groups(N);
  // phase 1 (independent of top_k)
  w.part = (float*)take((size_t)2 * G * 2 * B * 4);
  w.argpos = (int*)take((size_t)2 * G * B * 4);
  w.uop = (uint16_t*)take((size_t)2 * B * dk * 2);
  // phase 2
  w.theta = (float*)take((size_t)B * G * 4);
  w.uflag = (int*)take((size_t)B * 4);
  w.cv = (float*)take((size_t)B * kHpCap * 4);
  w.ci = (int64_t*)take((size_t)B * kHpCap * 8);
  w.cn = (int*)take((size_t)B * 4);
  w.flag = (int*)take(4);
  w.total = off + 256;
  return w;
}

}  // namespace hrec

using namespace hrec;

static int hp_check_args(const float* als_users, int64_t als_ld, int64_t n_als_rows, int als_width,
                         const float* tt_users, int64_t tt_ld, int tt_width, int n_users, const void* als_items,
                         const void* tt_items, int64_t n_items, int dk, const char* who) {
  HREC_REQUIRE(dk == 64 || dk == 128 || dk == 256, "%s: dk must be 64, 128 or 256 (got %d)", who, dk);
  HREC_REQUIRE(n_users >= 0 && n_users < 65536 && n_items >= 0 && n_items < 0x7fffffffll, "%s: bad shape", who);
  HREC_REQUIRE(als_width >= 0 && als_width <= dk && tt_width >= 0 && tt_width <= dk,
               "%s: user widths must be in [0, dk]", who);
  HREC_REQUIRE(als_ld >= als_width && tt_ld >= tt_width && n_als_rows >= 0, "%s: bad user row stride / count", who);
  HREC_REQUIRE(n_users == 0 || n_items == 0 || (als_users && tt_users && als_items && tt_items), "%s: null pointer",
               who);
  HREC_REQUIRE((((uintptr_t)als_items | (uintptr_t)tt_items) & 15) == 0, "%s: item operands must be 16-B aligned", who);
  return HREC_OK;
}

extern "C" size_t hrec_hybrid_prune_workspace_bytes(int n_users, int64_t n_items, int dk, int top_k) {
  const int B = n_users > 0 ? n_users : 0;
  const int64_t N = n_items > 0 ? n_items : 0;
  int kk = (int)(top_k < N ? top_k : N);
  kk = kk < 1 ? 1 : (kk > kHpMaxK ? kHpMaxK : kk);
  return hp_layout(nullptr, B, N, dk, kk).total;
}

extern "C" int hrec_hybrid_prune_minmax(const float* als_users, int64_t als_ld, const int64_t* als_rows,
                                        int64_t n_als_rows, int als_width, const float* tt_users, int64_t tt_ld,
                                        int tt_width, int n_users, const void* als_items, const void* tt_items,
                                        int64_t n_items, int dk, float* als_mm, float* tt_mm, void* workspace,
                                        size_t workspace_bytes, void* stream) {
  int rc = hp_check_args(als_users, als_ld, n_als_rows, als_width, tt_users, tt_ld, tt_width, n_users, als_items,
                         tt_items, n_items, dk, "hybrid_prune_minmax");
  if (rc) return rc;
  if (n_users == 0) return HREC_OK;
  HREC_REQUIRE(als_mm && tt_mm && workspace, "hybrid_prune_minmax: null min/max output or workspace");
  const size_t need = hrec_hybrid_prune_workspace_bytes(n_users, n_items, dk, 1);
  HREC_REQUIRE(workspace_bytes >= need, "hybrid_prune_minmax: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t s = as_stream(stream);
  const HpWs w = hp_layout((char*)workspace, n_users, n_items, dk, 1);
  if (n_items == 0)  // no items: min = +inf, max = -inf (hrec_hybrid_scores of an empty shard)
    return hrec_hybrid_scores(als_users, als_ld, als_rows, n_als_rows, als_width, tt_users, tt_ld, tt_width, n_users,
                              als_items, tt_items, 0, dk, nullptr, nullptr, 0, als_mm, tt_mm, w.part,
                              (size_t)2 * 2 * n_users * 4 + 256, stream);
  hipLaunchKernelGGL(hp_user_ops_kernel, dim3((unsigned)n_users, 2), dim3(256), 0, s, als_users, als_ld, als_rows,
                     n_als_rows, als_width, tt_users, tt_ld, tt_width, n_users, dk, w.uop);
  rc = check_launch("hp_user_ops_kernel");
  if (rc) return rc;
  return hybrid_scores_run(1 /* HS_PRUNE */, als_users, als_ld, als_rows, n_als_rows, als_width, tt_users, tt_ld,
                           tt_width, n_users, als_items, tt_items, n_items, dk, nullptr, nullptr, 0, als_mm, tt_mm,
                           w.part, w.argpos, s, w.uop);
}

// Phase 2 launches (a - c). local: the bound kernel reduces the extremes
// from phase 1's partials (written to als_mm_out / tt_mm_out) instead of
// reading them.
static int hp_phase2(bool local, int n_users, const void* als_items, const void* tt_items, int64_t n_items, int dk,
                     const float* als_mm, const float* tt_mm, float* als_mm_out, float* tt_mm_out, int als_wins,
                     int top_k, int64_t idx_offset, int64_t* out_idx, double* out_val, void* workspace,
                     hipStream_t s) {
  const int kk = (int)(top_k < n_items ? top_k : n_items);
  const HpWs w = hp_layout((char*)workspace, n_users, n_items, dk, kk);
  // src/hybrid_system.py:69 — strict '>' picks (0.8, 0.2), else (0.2, 0.8); the heavier model filters
  const double w0 = als_wins ? 0.8 : 0.2, w1 = als_wins ? 0.2 : 0.8;
  const int hm = als_wins ? 0 : 1;
  const int G = hs_groups(n_items);
  const uint16_t* ai = static_cast<const uint16_t*>(als_items);
  const uint16_t* ti = static_cast<const uint16_t*>(tt_items);
  // hp_bound_kernel's LDS slots hold kHpMaxGroups x 16 items: 16 per group = 4 tiles of 4 (HREC_HS_NI* builds)
  HREC_REQUIRE(hs_slice_tiles(dk) <= 4, "hybrid_prune: slice of %d tiles exceeds the bound kernel's 4",
               hs_slice_tiles(dk));
#define HREC_HP_BOUND(DK, L)                                                                                 \
  hipLaunchKernelGGL((hp_bound_kernel<DK, L>), dim3((unsigned)n_users), dim3(256), 0, s, w.part, w.argpos, G,        \
                     n_items, n_users, hm, als_mm, tt_mm, als_mm_out, tt_mm_out, w0, w1, kk, hs_slice_tiles(DK),   \
                     w.uop, ai, ti, w.theta, w.cn, w.uflag, w.flag)
  switch (dk) {
    case 64:
      if (local) HREC_HP_BOUND(64, true); else HREC_HP_BOUND(64, false);
      break;
    case 128:
      if (local) HREC_HP_BOUND(128, true); else HREC_HP_BOUND(128, false);
      break;
    default:
      if (local) HREC_HP_BOUND(256, true); else HREC_HP_BOUND(256, false);
      break;
  }
#undef HREC_HP_BOUND
  int rc = check_launch("hp_bound_kernel");
  if (rc) return rc;
  // b. the heavy model's scores, survivors of the per-group bounds: one
  //    block per item group (the bound is one LDS value per user), the
  //    phase-1 GEMM's tiling and k order (the same scores)
  const HsFilter f{w.theta, hm, kHpCap, w.cv, w.ci, w.cn};
  rc = hybrid_scores_run(2 /* HS_FILTER */, nullptr, 0, nullptr, 0, 0, nullptr, 0, 0, n_users, als_items, tt_items,
                         n_items, dk, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr, s, w.uop, &f);
  if (rc) return rc;
  // c. light scores + fusion of the survivors, exact top-k; the exact path in
  //    the same block for the users that need it
  const float* amm = local ? als_mm_out : als_mm;
  const float* tmm = local ? tt_mm_out : tt_mm;
#define HREC_HP_CAND(DK)                                                                                           \
  hipLaunchKernelGGL(hp_cand_topk_kernel<DK>, dim3((unsigned)n_users), dim3(512), 0, s, w.cn, kHpCap, w.cv, w.ci,   \
                     w.uflag, w.uop, hm, als_items, tt_items, n_items, n_users, amm, tmm, w0, w1, kk,              \
                     idx_offset, out_idx, out_val, w.flag)
  switch (dk) {
    case 64: HREC_HP_CAND(64); break;
    case 128: HREC_HP_CAND(128); break;
    default: HREC_HP_CAND(256); break;
  }
#undef HREC_HP_CAND
  return check_launch("hp_cand_topk_kernel");
}

extern "C" int hrec_hybrid_prune_topk(const float* als_users, int64_t als_ld, const int64_t* als_rows,
                                      int64_t n_als_rows, int als_width, const float* tt_users, int64_t tt_ld,
                                      int tt_width, int n_users, const void* als_items, const void* tt_items,
                                      int64_t n_items, int dk, const float* als_mm, const float* tt_mm, int als_wins,
                                      int top_k, int64_t idx_offset, int64_t* out_idx, double* out_val,
                                      void* workspace, size_t workspace_bytes, void* stream) {
  int rc = hp_check_args(als_users, als_ld, n_als_rows, als_width, tt_users, tt_ld, tt_width, n_users, als_items,
                         tt_items, n_items, dk, "hybrid_prune_topk");
  if (rc) return rc;
  HREC_REQUIRE(top_k >= 1 && top_k <= kHpMaxK, "hybrid_prune_topk: top_k must be in [1, %d] (larger: the unfused path)",
               kHpMaxK);
  if (n_users == 0 || n_items == 0) return HREC_OK;
  HREC_REQUIRE(als_mm && tt_mm && out_idx && out_val && workspace, "hybrid_prune_topk: null pointer");
  const size_t need = hrec_hybrid_prune_workspace_bytes(n_users, n_items, dk, top_k);
  HREC_REQUIRE(workspace_bytes >= need, "hybrid_prune_topk: workspace %zu < %zu", workspace_bytes, need);
  return hp_phase2(false, n_users, als_items, tt_items, n_items, dk, als_mm, tt_mm, nullptr, nullptr, als_wins, top_k,
                   idx_offset, out_idx, out_val, workspace, as_stream(stream));
}

extern "C" int hrec_hybrid_prune_local(const float* als_users, int64_t als_ld, const int64_t* als_rows,
                                       int64_t n_als_rows, int als_width, const float* tt_users, int64_t tt_ld,
                                       int tt_width, int n_users, const void* als_items, const void* tt_items,
                                       int64_t n_items, int dk, int als_wins, int top_k, int64_t idx_offset,
                                       float* als_mm, float* tt_mm, int64_t* out_idx, double* out_val,
                                       void* workspace, size_t workspace_bytes, void* stream) {
  int rc = hp_check_args(als_users, als_ld, n_als_rows, als_width, tt_users, tt_ld, tt_width, n_users, als_items,
                         tt_items, n_items, dk, "hybrid_prune_local");
  if (rc) return rc;
  HREC_REQUIRE(top_k >= 1 && top_k <= kHpMaxK, "hybrid_prune_local: top_k must be in [1, %d] (larger: the unfused path)",
               kHpMaxK);
  if (n_users == 0) return HREC_OK;
  HREC_REQUIRE(als_mm && tt_mm && workspace, "hybrid_prune_local: null pointer");
  if (n_items == 0)  // extremes of an empty shard; no top-k entries
    return hrec_hybrid_prune_minmax(als_users, als_ld, als_rows, n_als_rows, als_width, tt_users, tt_ld, tt_width,
                                    n_users, als_items, tt_items, 0, dk, als_mm, tt_mm, workspace, workspace_bytes,
                                    stream);
  HREC_REQUIRE(out_idx && out_val, "hybrid_prune_local: null output");
  const size_t need = hrec_hybrid_prune_workspace_bytes(n_users, n_items, dk, top_k);
  HREC_REQUIRE(workspace_bytes >= need, "hybrid_prune_local: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t s = as_stream(stream);
  const HpWs w = hp_layout((char*)workspace, n_users, n_items, dk, 1);
  hipLaunchKernelGGL(hp_user_ops_kernel, dim3((unsigned)n_users, 2), dim3(256), 0, s, als_users, als_ld, als_rows,
                     n_als_rows, als_width, tt_users, tt_ld, tt_width, n_users, dk, w.uop);
  rc = check_launch("hp_user_ops_kernel");
  if (rc) return rc;
  // phase 1 without its min / max reduce launch (the bound kernel folds it)
  rc = hybrid_scores_run(1 /* HS_PRUNE */, als_users, als_ld, als_rows, n_als_rows, als_width, tt_users, tt_ld,
                         tt_width, n_users, als_items, tt_items, n_items, dk, nullptr, nullptr, 0, nullptr, nullptr,
                         w.part, w.argpos, s, w.uop);
  if (rc) return rc;
  return hp_phase2(true, n_users, als_items, tt_items, n_items, dk, nullptr, nullptr, als_mm, tt_mm, als_wins, top_k,
                   idx_offset, out_idx, out_val, workspace, s);
}

#ifdef HREC_HP_STAMPS
extern "C" int hrec_debug_hp_stamps(unsigned long long* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_hp_stamps), sizeof(g_hp_stamps)) == hipSuccess ? 0 : -2;
}
#endif

extern "C" int hrec_hybrid_prune_survivors(const void* workspace, int n_users, int64_t n_items, int dk, int top_k,
                                           int32_t* out, void* stream) {
  HREC_REQUIRE(workspace && out && n_users >= 0 && n_items >= 0, "hybrid_prune_survivors: bad argument");
  int kk = (int)(top_k < n_items ? top_k : n_items);
  kk = kk < 1 ? 1 : (kk > kHpMaxK ? kHpMaxK : kk);
  const HpWs w = hp_layout((char*)workspace, n_users, n_items, dk, kk);
  if (n_users > 0 &&
      hipMemcpyAsync(out, w.cn, (size_t)n_users * 4, hipMemcpyDeviceToDevice, as_stream(stream)) != hipSuccess)
    return check_launch("hybrid_prune_survivors: copy");
  return HREC_OK;
}

extern "C" int hrec_hybrid_prune_fallback_taken(const void* workspace, int n_users, int64_t n_items, int dk,
                                                int top_k, int* out, void* stream) {
  HREC_REQUIRE(workspace && out && n_users >= 0 && n_items >= 0, "hybrid_prune_fallback_taken: bad argument");
  int kk = (int)(top_k < n_items ? top_k : n_items);
  kk = kk < 1 ? 1 : (kk > kHpMaxK ? kHpMaxK : kk);
  const HpWs w = hp_layout((char*)workspace, n_users, n_items, dk, kk);
  if (hipMemcpyAsync(out, w.flag, 4, hipMemcpyDeviceToDevice, as_stream(stream)) != hipSuccess)
    return check_launch("hybrid_prune_fallback_taken: copy");
  return HREC_OK;
}
