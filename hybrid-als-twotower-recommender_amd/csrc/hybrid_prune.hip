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
//     bf16 operands; both GEMMs (hyb_scores_kernel, mode HS_PRUNE: no stores)
//     -> per-user min / max of both rows, and per item group (block) the 16-NI
//     item slice holding the group's maximum;
//   [the caller all-reduces the min / max across item shards (C2)]
//   phase 2 (hrec_hybrid_prune_topk):
//     a. bound: per user, the slices of the 2k groups with the largest maxima
//        of the HEAVY model (weight 0.8) — 8 or 16 distinct items each; their
//        fused scores, from both dot products recomputed in f32 and lowered by
//        the rounding bound (|sum - mfma| <= 2^-15 sum|p| at dk <= 256), give
//        tau <= the k-th best fused score of the shard. Any item of the top k
//        has w_h h_n + w_l l_n >= tau with l_n <= the light row's max scaled,
//        hence its heavy raw score >= theta (computed in f64, lowered by a
//        relative margin);
//     b. the heavy model's GEMM alone with the survivor filter score >= theta
//        (dot_res_kernel FILTER, K8): the few survivors (item ids + exact
//        heavy scores) per user;
//     c. each survivor's light score with the same bf16 MFMA k order (A =
//        the gathered item rows, B = the user row), the fused score with
//        fuse_rows_kernel's arithmetic (ALS branch f64, two-tower f32, numpy
//        1.21 promotion), then the exact stable top-k (ties -> smaller item);
//     d. (gated on the device flag: list overflow, fewer than k survivors or
//        non-finite extremes) the exact unfused path — both score matrices
//        into the workspace + hrec_fuse_rows_topk's segment path — so no host
//        round trip is needed and a batch can be captured as one HIP graph.
// Bit-identical to hrec_hybrid_scores + hrec_fuse_rows_topk: every score is
// the same MFMA chain and every fused score the same arithmetic.
#include <float.h>
#include <math.h>

#include "common.h"

namespace hrec {

typedef float hp_f4 __attribute__((ext_vector_type(4)));
typedef __bf16 hp_bf8 __attribute__((ext_vector_type(8)));

union HpFrag {
  int4 i;
  hp_f4 f;
};

constexpr int kHpCap = 8192;      // survivors per user (expected: a few hundred)
constexpr int kHpMaxK = 8;        // top_k handled here (kFuseK of the exact path)
constexpr int kHpMaxGroups = 16;  // heavy-model groups whose max slices seed the bound

// f32 -> bf16 bits, round to nearest even (NaN stays NaN): hrec_f32_to_bf16.
__device__ __forceinline__ uint32_t hp_bf16(float v) {
  const uint32_t x = __float_as_uint(v);
  if ((x & 0x7fffffffu) > 0x7f800000u) return (x >> 16) | 0x40u;
  return (x + 0x7fffu + ((x >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ float hp_f(uint32_t bits16) { return __uint_as_float(bits16 << 16); }

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The scaler coefficients of fuse_rows_kernel (sklearn MinMaxScaler: ALS in
// f64, two-tower in f32; range < 10 eps -> 1).
struct HpScale {
  double ascale, amin_;
  float tscale, tmin_;
};
__device__ __forceinline__ HpScale hp_scale(float amin, float amax, float tmin, float tmax) {
#pragma clang fp contract(off)
  HpScale s;
  double arange = (double)amax - (double)amin;
  if (arange < 10.0 * DBL_EPSILON) arange = 1.0;
  s.ascale = 1.0 / arange;
  s.amin_ = 0.0 - (double)amin * s.ascale;
  float trange = tmax - tmin;
  if (trange < 10.0f * FLT_EPSILON) trange = 1.0f;
  s.tscale = 1.0f / trange;
  s.tmin_ = 0.0f - tmin * s.tscale;
  return s;
}
__device__ __forceinline__ double hp_fuse(const HpScale& s, float a, float t, double w0, double w1) {
#pragma clang fp contract(off)
  const double an = (double)a * s.ascale + s.amin_;
  const float tn = t * s.tscale + s.tmin_;
  return w0 * an + w1 * (double)tn;
}

// 1. bf16 user operands [2][B][dk]: the ALS rows gathered by als_rows (a row
// outside [0, n_als_rows) reads as NaN, as hyb_scores_kernel stages it) and
// the two-tower rows, columns >= width zero — hyb_scores_kernel's staging.
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

// 2a. The bound: one wave per user (no block barriers).
template <int DK>
__global__ __launch_bounds__(256) void hp_bound_kernel(const float* __restrict__ part, const int* __restrict__ argpos,
                                                       int G, int64_t N, int B, int hm, const float* __restrict__ als_mm,
                                                       const float* __restrict__ tt_mm, double w0, double w1, int kk,
                                                       int slice_ni, const uint16_t* __restrict__ uop,
                                                       const uint16_t* __restrict__ als_items,
                                                       const uint16_t* __restrict__ tt_items,
                                                       float* __restrict__ theta, int* __restrict__ flag) {
#pragma clang fp contract(off)
  constexpr int kSlots = kHpMaxGroups * 16;  // <= 16 groups x (4 NI <= 16) items
  __shared__ float smax[4][128];
  __shared__ int sitem[4][kSlots];
  __shared__ double sfl[4][kSlots];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = blockIdx.x * 4 + wv;
  if (b >= B) return;  // wave-uniform
  const float amin = als_mm[b], amax = als_mm[B + b], tmin = tt_mm[b], tmax = tt_mm[B + b];
  if (!(isfinite(amin) && isfinite(amax) && isfinite(tmin) && isfinite(tmax))) {
    // NaN / infinite scores (an unknown user row, non-finite vectors): the
    // exact path ranks them
    if (lane == 0) {
      theta[b] = __builtin_nanf("");
      *flag = 1;
    }
    return;
  }
  const HpScale sc = hp_scale(amin, amax, tmin, tmax);
  const int64_t per = ((N + G - 1) / G + 15) / 16 * 16;  // hyb_scores_kernel's group range
  // group maxima of the heavy model and their rank (value desc, group asc)
  for (int gi = lane; gi < 128; gi += 64) {
    float v = -INFINITY;
    if (gi < G && argpos[((int64_t)hm * G + gi) * B + b] >= 0) v = part[(((int64_t)hm * G + gi) * 2 + 1) * B + b];
    smax[wv][gi] = v;
  }
  wave_sync_lds();
  const int M = 2 * kk < kHpMaxGroups ? 2 * kk : kHpMaxGroups;
  const int per_g = 4 * slice_ni;
  for (int s = lane; s < kSlots; s += 64) sitem[wv][s] = -1;
  wave_sync_lds();
  for (int gi = lane; gi < G; gi += 64) {
    const float v = smax[wv][gi];
    if (v == -INFINITY) continue;
    int rank = 0;
    for (int q = 0; q < G; ++q) {
      const float o = smax[wv][q];
      rank += (o > v || (o == v && q < gi)) ? 1 : 0;
    }
    if (rank < M) {
      const int pos = argpos[((int64_t)hm * G + gi) * B + b];
      const int64_t jb = (int64_t)(pos >> 2) * 16;
      const int g = pos & 3;
      const int64_t i1 = (int64_t)gi * per + per < N ? (int64_t)gi * per + per : N;
      for (int t = 0; t < slice_ni; ++t)
        for (int r = 0; r < 4; ++r) {
          const int64_t j = jb + 16 * t + 4 * g + r;
          sitem[wv][rank * per_g + 4 * t + r] = j < i1 ? (int)j : -1;
        }
    }
  }
  wave_sync_lds();
  // both dot products of every seed item in f32 (products exact), lowered by
  // the rounding bound to a valid lower bound of its fused score
  const uint16_t* uh = uop + ((int64_t)hm * B + b) * DK;
  const uint16_t* ul = uop + ((int64_t)(1 - hm) * B + b) * DK;
  const uint16_t* vh_base = hm ? tt_items : als_items;
  const uint16_t* vl_base = hm ? als_items : tt_items;
  const int n_slots = M * per_g;
  for (int s = lane; s < n_slots; s += 64) {
    const int j = sitem[wv][s];
    double fl = -INFINITY;
    if (j >= 0) {
      const uint16_t* vh = vh_base + (int64_t)j * DK;
      const uint16_t* vl = vl_base + (int64_t)j * DK;
      float ah = 0.f, al = 0.f, sh = 0.f, sl = 0.f;
      for (int c0 = 0; c0 < DK; c0 += 8) {
        const uint4 xh = *reinterpret_cast<const uint4*>(vh + c0);
        const uint4 xl = *reinterpret_cast<const uint4*>(vl + c0);
        const uint4 yh = *reinterpret_cast<const uint4*>(uh + c0);
        const uint4 yl = *reinterpret_cast<const uint4*>(ul + c0);
        const uint32_t ph[4] = {xh.x, xh.y, xh.z, xh.w}, pl[4] = {xl.x, xl.y, xl.z, xl.w};
        const uint32_t qh[4] = {yh.x, yh.y, yh.z, yh.w}, ql[4] = {yl.x, yl.y, yl.z, yl.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float h0 = hp_f(ph[e] & 0xffffu) * hp_f(qh[e] & 0xffffu), h1 = hp_f(ph[e] >> 16) * hp_f(qh[e] >> 16);
          const float l0 = hp_f(pl[e] & 0xffffu) * hp_f(ql[e] & 0xffffu), l1 = hp_f(pl[e] >> 16) * hp_f(ql[e] >> 16);
          ah += h0;
          ah += h1;
          al += l0;
          al += l1;
          sh += fabsf(h0) + fabsf(h1);
          sl += fabsf(l0) + fabsf(l1);
        }
      }
      // |f32 sum - exact| and |MFMA - exact| are each <= 2^-16 sum|p| (n <= 256)
      const double mh = 0x1p-15 * (double)sh * 1.001, ml = 0x1p-15 * (double)sl * 1.001;
      const float a = hm ? al : ah, t = hm ? ah : al;
      const double ma = hm ? ml : mh, mt = hm ? mh : ml;
      const double f = hp_fuse(sc, a, t, w0, w1);
      // the fused score moves by at most w0 ascale ma + w1 (tscale mt + the f32 rounding of tn)
      const double err = w0 * sc.ascale * ma + w1 * ((double)sc.tscale * mt * 1.001 + 1e-6) + 1e-12;
      if (f == f) fl = f - err;
    }
    sfl[wv][s] = fl;
  }
  wave_sync_lds();
  // tau = the kk-th largest lower bound (the seed items are distinct)
  double tau = -INFINITY;
  for (int s = lane; s < n_slots; s += 64) {
    const double v = sfl[wv][s];
    if (v == -INFINITY) continue;
    int rank = 0;
    for (int q = 0; q < n_slots; ++q) {
      const double o = sfl[wv][q];
      rank += (o > v || (o == v && q < s)) ? 1 : 0;
    }
    if (rank == kk - 1) tau = v;
  }
  // the lane that found it: broadcast by a max over the wave (-inf elsewhere)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) tau = fmax(tau, __shfl_xor(tau, off, kWave));
  if (lane != 0) return;
  float th = -INFINITY;
  if (tau > -INFINITY) {
    if (hm == 0) {  // heavy = ALS (w0): a_n >= (tau - w1 * max t_n) / w0
      const float tn_max = tmax * sc.tscale + sc.tmin_;
      const double hn = (tau - w1 * (double)tn_max) / w0 - 1e-9;
      double x = (hn - sc.amin_) / sc.ascale;
      x -= 1e-6 * (fabs(x) + ((double)amax - (double)amin));
      th = (float)x;
      if ((double)th > x) th = nextafterf(th, -INFINITY);
    } else {        // heavy = two-tower (w1): t_n >= (tau - w0 * max a_n) / w1
      const double an_max = (double)amax * sc.ascale + sc.amin_;
      const double hn = (tau - w0 * an_max) / w1 - 1e-9;
      double x = (hn - (double)sc.tmin_) / (double)sc.tscale;
      x -= 1e-6 * (fabs(x) + ((double)tmax - (double)tmin));
      th = (float)x;
      if ((double)th > x) th = nextafterf(th, -INFINITY);
    }
  }
  theta[b] = th;
}

// 2b'. list checks: overflow (cn > cap) or fewer survivors than the top-k
// needs (only with NaN scores) -> the exact fallback.
__global__ void hp_check_kernel(const int* __restrict__ cn, int B, int cap, int need, int* __restrict__ flag) {
  for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < B; b += gridDim.x * blockDim.x)
    if (cn[b] > cap || cn[b] < need) *flag = 1;
}

// 2c. Survivors: light scores (MFMA over 16 gathered items against the
// user row), fused scores. One wave per 16 survivors of user blockIdx.y.
template <int DK>
__global__ __launch_bounds__(256) void hp_cand_kernel(const int* __restrict__ cn, int cap, const float* __restrict__ cv,
                                                      const int64_t* __restrict__ ci, const uint16_t* __restrict__ ul_base,
                                                      const void* __restrict__ light_items, int64_t N, int B, int hm,
                                                      const float* __restrict__ als_mm, const float* __restrict__ tt_mm,
                                                      double w0, double w1, double* __restrict__ fv) {
  constexpr int KS = DK / 32;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int b = blockIdx.y;
  int nb = cn[b];
  nb = nb < cap ? nb : cap;
  if (16 * (blockIdx.x * 4 + wv) >= nb) return;  // wave-uniform
  const HpScale sc = hp_scale(als_mm[b], als_mm[B + b], tt_mm[b], tt_mm[B + b]);
  const char* ur = reinterpret_cast<const char*>(ul_base + (int64_t)b * DK);
  HpFrag uf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) uf[ks].i = *reinterpret_cast<const int4*>(ur + 16 * g + 64 * ks);
  const char* vbase = static_cast<const char*>(light_items);
  for (int q = blockIdx.x * 4 + wv; 16 * q < nb; q += gridDim.x * 4) {
    const int pos = 16 * q + c;
    const int64_t item = pos < nb ? ci[(int64_t)b * cap + pos] : -1;
    // survivors are arbitrary rows: 64-bit addresses (a buffer resource spans
    // at most 4 GiB); a padding slot reads row 0 and its result is dropped
    const char* row = vbase + (item >= 0 && item < N ? item : 0) * (int64_t)(DK * 2);
    HpFrag it[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) it[ks].i = *reinterpret_cast<const int4*>(row + 16 * g + 64 * ks);
    hp_f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)  // A = items, B = users: the k order of hyb_scores_kernel / dot_res_kernel
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(hp_bf8, it[ks].i),
                                                    __builtin_bit_cast(hp_bf8, uf[ks].i), acc, 0, 0, 0);
    if (c == 0) {  // C/D: lane (g, c) holds rows 4 g + r (the survivors) of column c (every column is the user)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * q + 4 * g + r;
        if (p < nb) {
          const float h = cv[(int64_t)b * cap + p], l = acc[r];
          fv[(int64_t)b * cap + p] = hm ? hp_fuse(sc, l, h, w0, w1) : hp_fuse(sc, h, l, w0, w1);
        }
      }
    }
  }
}

struct HpWs {
  float* part;
  int* argpos;
  uint16_t* uop;
  float* theta;
  float* cv;
  int64_t* ci;
  int* cn;
  int* flag;
  double* fv;
  char* tws;
  float* fb;
  char* fws;
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
  w.theta = (float*)take((size_t)B * 4);
  w.cv = (float*)take((size_t)B * kHpCap * 4);
  w.ci = (int64_t*)take((size_t)B * kHpCap * 8);
  w.cn = (int*)take((size_t)B * 4);
  w.flag = (int*)take(4);
  w.fv = (double*)take((size_t)B * kHpCap * 8);
  w.tws = take(topk_ws_bytes(B, kHpCap, kk, 8));
  w.fb = (float*)take((size_t)2 * B * N * 4);  // exact fallback: both score matrices
  w.fws = take(fuse_rows_exact_ws_bytes(B, N, kk));
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
  hipLaunchKernelGGL(hp_user_ops_kernel, dim3((unsigned)n_users, 2), dim3(256), 0, s, als_users, als_ld, als_rows,
                     n_als_rows, als_width, tt_users, tt_ld, tt_width, n_users, dk, w.uop);
  rc = check_launch("hp_user_ops_kernel");
  if (rc) return rc;
  if (n_items == 0)  // no items: min = +inf, max = -inf (hrec_hybrid_scores of an empty shard)
    return hrec_hybrid_scores(als_users, als_ld, als_rows, n_als_rows, als_width, tt_users, tt_ld, tt_width, n_users,
                              als_items, tt_items, 0, dk, nullptr, nullptr, 0, als_mm, tt_mm, w.part,
                              (size_t)2 * 2 * n_users * 4 + 256, stream);
  return hybrid_scores_run(1 /* HS_PRUNE */, als_users, als_ld, als_rows, n_als_rows, als_width, tt_users, tt_ld,
                           tt_width, n_users, als_items, tt_items, n_items, dk, nullptr, nullptr, 0, als_mm, tt_mm,
                           w.part, w.argpos, nullptr, s);
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
  hipStream_t s = as_stream(stream);
  const int kk = (int)(top_k < n_items ? top_k : n_items);
  const HpWs w = hp_layout((char*)workspace, n_users, n_items, dk, kk);
  // src/hybrid_system.py:69 — strict '>' picks (0.8, 0.2), else (0.2, 0.8); the heavier model filters
  const double w0 = als_wins ? 0.8 : 0.2, w1 = als_wins ? 0.2 : 0.8;
  const int hm = als_wins ? 0 : 1;
  const int G = hs_groups(n_items);
  if (hipMemsetAsync(w.flag, 0, 4, s) != hipSuccess || hipMemsetAsync(w.cn, 0, (size_t)n_users * 4, s) != hipSuccess)
    return check_launch("hybrid_prune_topk: memset");
  const dim3 gb((unsigned)((n_users + 3) / 4));
  const uint16_t* ai = static_cast<const uint16_t*>(als_items);
  const uint16_t* ti = static_cast<const uint16_t*>(tt_items);
#define HREC_HP_BOUND(DK)                                                                                        \
  hipLaunchKernelGGL(hp_bound_kernel<DK>, gb, dim3(256), 0, s, w.part, w.argpos, G, n_items, n_users, hm, als_mm, \
                     tt_mm, w0, w1, kk, hs_slice_tiles(DK), w.uop, ai, ti, w.theta, w.flag)
  switch (dk) {
    case 64: HREC_HP_BOUND(64); break;
    case 128: HREC_HP_BOUND(128); break;
    default: HREC_HP_BOUND(256); break;
  }
#undef HREC_HP_BOUND
  rc = check_launch("hp_bound_kernel");
  if (rc) return rc;
  // b. the heavy model's scores, survivors of theta
  const uint16_t* uh = w.uop + (size_t)hm * n_users * dk;
  const uint16_t* ul = w.uop + (size_t)(1 - hm) * n_users * dk;
  rc = dot_filter_run(uh, n_users, hm ? tt_items : als_items, n_items, dk, 1, w.theta, kHpCap, w.cv, w.ci, w.cn, s);
  if (rc) return rc;
  hipLaunchKernelGGL(hp_check_kernel, dim3(64), dim3(256), 0, s, w.cn, n_users, kHpCap, kk, w.flag);
  rc = check_launch("hp_check_kernel");
  if (rc) return rc;
  // c. light scores + fusion of the survivors, exact top-k
  const dim3 gc(8, (unsigned)n_users);
#define HREC_HP_CAND(DK)                                                                                          \
  hipLaunchKernelGGL(hp_cand_kernel<DK>, gc, dim3(256), 0, s, w.cn, kHpCap, w.cv, w.ci, ul, hm ? als_items : tt_items, \
                     n_items, n_users, hm, als_mm, tt_mm, w0, w1, w.fv)
  switch (dk) {
    case 64: HREC_HP_CAND(64); break;
    case 128: HREC_HP_CAND(128); break;
    default: HREC_HP_CAND(256); break;
  }
#undef HREC_HP_CAND
  rc = check_launch("hp_cand_kernel");
  if (rc) return rc;
  rc = topk_rows<double>(w.fv, n_users, kHpCap, kHpCap, kk, out_idx, out_val, w.tws, (size_t)1 << 62, s, w.ci, w.cn);
  if (rc) return rc;
  // d. exact fallback, gated on the flag (no host round trip)
  rc = hybrid_scores_run(2 /* HS_GATED */, als_users, als_ld, als_rows, n_als_rows, als_width, tt_users, tt_ld,
                         tt_width, n_users, als_items, tt_items, n_items, dk, w.fb, w.fb + (size_t)n_users * n_items,
                         n_items, nullptr, nullptr, nullptr, nullptr, w.flag, s);
  if (rc) return rc;
  rc = fuse_rows_exact(w.fb, w.fb + (size_t)n_users * n_items, n_users, n_items, n_items, als_mm, tt_mm, w0, w1, kk,
                       out_idx, out_val, w.fws, s, w.flag);
  if (rc) return rc;
  return offset_ids(out_idx, (int64_t)n_users * kk, idx_offset, s);
}

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
