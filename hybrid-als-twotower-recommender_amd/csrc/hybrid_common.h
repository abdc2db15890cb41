// Device helpers shared by the pruned hybrid top-k kernels (csrc/hybrid_prune.hip,
// bf16 c5 path; csrc/hybrid_exact.hip, exact c2 path): the fusion arithmetic of
// fuse_rows_kernel (src/hybrid_system.py:57-75), the top-k order of
// score.hip's better() (sorted(..., reverse=True) over the reference's
// candidate order, src/hybrid_system.py:108) and 64-bit lane moves.
#pragma once

#include <float.h>
#include <math.h>

#include "common.h"

namespace hrec {

typedef float hp_f4 __attribute__((ext_vector_type(4)));

// f32 -> bf16 bits, round to nearest even (NaN stays NaN): hrec_f32_to_bf16.
__device__ __forceinline__ uint32_t hp_bf16(float v) {
  const uint32_t x = __float_as_uint(v);
  if ((x & 0x7fffffffu) > 0x7f800000u) return (x >> 16) | 0x40u;
  return (x + 0x7fffu + ((x >> 16) & 1u)) >> 16;
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
// Non-decreasing in a and in t (positive scales and weights, rounding is
// monotone): the fused score of an upper bound of (a, t) bounds the item's.
__device__ __forceinline__ double hp_fuse(const HpScale& s, float a, float t, double w0, double w1) {
#pragma clang fp contract(off)
  const double an = (double)a * s.ascale + s.amin_;
  const float tn = t * s.tscale + s.tmin_;
  return w0 * an + w1 * (double)tn;
}

// Order of the fused top-k (score.hip's better()): larger first, equal ->
// smaller item id, NaN last.
__device__ __forceinline__ bool hp_better(double va, int64_t ia, double vb, int64_t ib) {
  const bool na = va != va, nb = vb != vb;
  if (na || nb) return !na && nb ? true : (na && nb ? ia < ib : false);
  return va > vb || (va == vb && ia < ib);
}

// hp_better's order as one unsigned key (larger = better; ties -> the smaller
// item): 0 = an empty slot (idx INT64_MAX), 1 = NaN, numbers above by their
// ordered bits (-0 folded into +0, equal values share a key).
__device__ __forceinline__ uint64_t hp_order_key(double v, int64_t idx) {
  const double z = v + 0.0;  // -0 + 0 = +0
  const uint64_t u = (uint64_t)__double_as_longlong(z);
  const uint64_t ord = (u >> 63) ? ~u : (u | 0x8000000000000000ull);
  return idx == INT64_MAX ? 0ull : (v != v ? 1ull : ord);
}

// 64-bit moves across lanes: DPP (CTRL: gfx9 dpp_ctrl, all sources valid)
// and readlane, as two 32-bit halves.
template <int CTRL, typename T>
__device__ __forceinline__ T hp_dpp64(T x) {
  static_assert(sizeof(T) == 8, "64-bit values");
  uint64_t u;
  __builtin_memcpy(&u, &x, 8);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xf, 0xf, false);
  u = ((uint64_t)hi << 32) | lo;
  T r;
  __builtin_memcpy(&r, &u, 8);
  return r;
}
template <int CTRL>
__device__ __forceinline__ float hp_dpp32(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, false));
}
// lane ^ 16 / lane ^ 32 by v_permlane16_swap / v_permlane32_swap (see
// csrc/hybrid_scores.hip hs_xor16)
__device__ __forceinline__ float hp_xor16(float x) {
  const uint32_t u = __float_as_uint(x);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]);
}
__device__ __forceinline__ float hp_xor32(float x) {
  const uint32_t u = __float_as_uint(x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}
template <typename T>
__device__ __forceinline__ T hp_readlane64(T x, int src) {
  static_assert(sizeof(T) == 8, "64-bit values");
  uint64_t u;
  __builtin_memcpy(&u, &x, 8);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, src);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), src);
  u = ((uint64_t)hi << 32) | lo;
  T r;
  __builtin_memcpy(&r, &u, 8);
  return r;
}

__device__ __forceinline__ float hp_pick(const hp_f4& a, int r) {
  return r == 0 ? a[0] : (r == 1 ? a[1] : (r == 2 ? a[2] : a[3]));
}

// The wave's best (bv, bi) into every lane (empty slots: bi == INT64_MAX,
// worse than everything): the order as one integer key per entry, reduced
// by DPP within each 16-lane row (quad swaps, half-row and row mirrors:
// register moves, no LDS round trip) and across the 4 rows by readlanes.
__device__ __forceinline__ void hp_wave_best(double& bv, int64_t& bi) {
  uint64_t k = hp_order_key(bv, bi);
  int64_t i = bi;
  double v = bv;
  auto fold = [&](uint64_t ok, int64_t oi, double ov) {
    const bool tk = (ok > k) | ((ok == k) & (oi < i));
    k = tk ? ok : k;
    i = tk ? oi : i;
    v = tk ? ov : v;
  };
  fold(hp_dpp64<0xB1>(k), hp_dpp64<0xB1>(i), hp_dpp64<0xB1>(v));     // quad_perm [1,0,3,2]
  fold(hp_dpp64<0x4E>(k), hp_dpp64<0x4E>(i), hp_dpp64<0x4E>(v));     // quad_perm [2,3,0,1]
  fold(hp_dpp64<0x141>(k), hp_dpp64<0x141>(i), hp_dpp64<0x141>(v));  // row_half_mirror
  fold(hp_dpp64<0x140>(k), hp_dpp64<0x140>(i), hp_dpp64<0x140>(v));  // row_mirror
  uint64_t bk = hp_readlane64(k, 0);
  int64_t bi2 = hp_readlane64(i, 0);
  double bv2 = hp_readlane64(v, 0);
#pragma unroll
  for (int r = 1; r < 4; ++r) {
    const uint64_t ok = hp_readlane64(k, 16 * r);
    const int64_t oi = hp_readlane64(i, 16 * r);
    const double ov = hp_readlane64(v, 16 * r);
    const bool tk = (ok > bk) | ((ok == bk) & (oi < bi2));
    bk = tk ? ok : bk;
    bi2 = tk ? oi : bi2;
    bv2 = tk ? ov : bv2;
  }
  bv = bv2;
  bi = bi2;
}

// A lane's sorted best KK (value, item) entries (empty: INT64_MAX).
template <int KK>
struct HpList {
  double v[KK];
  int64_t i[KK];
  __device__ __forceinline__ void reset() {
#pragma unroll
    for (int j = 0; j < KK; ++j) {
      v[j] = 0.0;
      i[j] = INT64_MAX;
    }
  }
  __device__ __forceinline__ void insert(double xv, int64_t xi) {
#pragma unroll
    for (int j = 0; j < KK; ++j) {  // compare-exchange chain (sorted list)
      const bool sw = i[j] == INT64_MAX || hp_better(xv, xi, v[j], i[j]);
      const double tv = v[j];
      const int64_t ti = i[j];
      v[j] = sw ? xv : tv;
      i[j] = sw ? xi : ti;
      xv = sw ? tv : xv;
      xi = sw ? ti : xi;
    }
  }
  // the wave's kk best entries, rank r into (rv[r], ri[r]) of lane 0; the
  // lanes' lists lose them (called wave-uniformly)
  __device__ __forceinline__ void wave_top(int kk, int lane, double* rv, int64_t* ri) {
    for (int r = 0; r < kk; ++r) {
      double bv = v[0];
      int64_t bi = i[0];
      hp_wave_best(bv, bi);
      if (lane == 0) {
        rv[r] = bv;
        ri[r] = bi;
      }
      if (bi != INT64_MAX && i[0] == bi) {  // the (unique) owner pops its head
#pragma unroll
        for (int j = 0; j + 1 < KK; ++j) {
          v[j] = v[j + 1];
          i[j] = i[j + 1];
        }
        i[KK - 1] = INT64_MAX;
      }
    }
  }
};

}  // namespace hrec
