// K2: ALS scoring (Spark ALSModel.transform, JVM-exact f32 chain),
// generic stable top-k (the reference's sorted(..., reverse=True)[:k]),
// K9: hybrid min-max fusion (src/hybrid_system.py:57-75) + top-k (:108).
#include <float.h>

#include "common.h"

namespace hrec {

#ifndef HREC_SCORE_PAIR_STORE
#define HREC_SCORE_PAIR_STORE 1  // full-row JVM-exact scores: 8-B stores of item pairs
#endif
constexpr int kScoreKMax = 256;  // widest factor row (rank 256)

// --------------------------------------------------------------- ALS score
// One thread per item; UB users per block row held in LDS (broadcast reads).
// The item matrix is stored transposed [kp][ld] so every c-step is one
// coalesced 1-KiB read per wave. Sequential c order, product rounded, sum
// rounded: Spark's `dotProduct += featuresA(i) * featuresB(i)` on floats.
template <int UB>
__global__ __launch_bounds__(256) void als_score_kernel(const float* __restrict__ U,
                                                        const int64_t* __restrict__ user_rows, int n_users,
                                                        const float* __restrict__ Vt, int64_t ld,
                                                        const int64_t* __restrict__ item_rows,
                                                        int64_t n_items, int k, int kp,
                                                        float* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ float ush[UB][kScoreKMax];
  __shared__ int uok[UB];
  const int b0 = blockIdx.y * UB;
  for (int t = threadIdx.x; t < UB * kp; t += blockDim.x) {
    const int b = t / kp, c = t % kp;
    const int64_t ur = (b0 + b < n_users) ? user_rows[b0 + b] : -1;
    ush[b][c] = ur >= 0 ? U[ur * kp + c] : 0.f;
    if (c == 0) uok[b] = ur >= 0;
  }
  __syncthreads();
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_items) return;
  const int64_t ir = item_rows ? item_rows[j] : j;
  float acc[UB];
#pragma unroll
  for (int b = 0; b < UB; ++b) acc[b] = 0.f;
  if (ir >= 0) {
    const float* __restrict__ v = Vt + ir;
    for (int c = 0; c < k; ++c) {
      const float vc = v[(int64_t)c * ld];
#pragma unroll
      for (int b = 0; b < UB; ++b) {
        const float prod = ush[b][c] * vc;
        acc[b] = acc[b] + prod;
      }
    }
  }
  const float qnan = __builtin_nanf("");
#pragma unroll
  for (int b = 0; b < UB; ++b) {
    if (b0 + b < n_users) out[(int64_t)(b0 + b) * n_items + j] = (ir >= 0 && uok[b]) ? acc[b] : qnan;
  }
}


// Fast path of K2 for whole item ranges (no item_rows gather): 4 items per
// thread (two float2 loads of the transposed item matrix per rank step),
// UB users per block kept TRANSPOSED in LDS (one ds_read_b128 feeds 4 users),
// packed f32 multiply + add (v_pk_mul_f32 / v_pk_add_f32; contraction off so
// every product and sum is rounded exactly like the JVM loop).
// FILTER: instead of writing the scores, append (score, item) pairs with
// score >= thr[b] to a per-user candidate list (wave-aggregated atomics).
typedef float f2v __attribute__((ext_vector_type(2)));
typedef int i4v __attribute__((ext_vector_type(4)));
// buffer_load_dwordx2 ... offen (raw: base + voffset, range-checked)
__device__ f2v rbuf_load_f2(i4v rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v2f32");

template <int UB, bool FILTER>
__global__ __launch_bounds__(256) void als_score_fast_kernel(
    const float* __restrict__ U, const int64_t* __restrict__ user_rows, int n_users,
    const float* __restrict__ Vt, int64_t ld, int64_t n_items, int k, int kp, float* __restrict__ out,
    const float* __restrict__ thr, int thr_stride, int cap, float* __restrict__ cand_v,
    int64_t* __restrict__ cand_i, int* __restrict__ cand_n, int* __restrict__ overflow) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float us[kScoreKMax + 1][UB];  // + the row read ahead past the end
  __shared__ int uok[UB];
  // grid: x = user group (fastest-varying), y = 1024-item slice, so the
  // blocks of one item slice are dispatched back to back and share it in L2
  const int b0 = blockIdx.x * UB;
  const int64_t j0 = (int64_t)blockIdx.y * 1024 + 2 * threadIdx.x;
  const int64_t j1 = j0 + 512;
  // Rank-step c reads row c of Vt through a raw buffer resource spanning
  // [0, ld) of that row (rows c >= k span nothing): columns past the row end
  // read as zero without a branch, and rank steps c + 1 ... c + P - 1 are
  // already in flight while step c computes. ld is even, so both items of a
  // pair are in range together; items in [n_items, ld) are dropped below.
  constexpr int P = 4;
  const uint64_t vbase = (uint64_t)Vt;
  const int rec = (int)(ld * 4);
  auto rsrc_of = [&](int c) {
    const uint64_t a = vbase + (uint64_t)c * (uint64_t)ld * 4u;
    i4v r;
    r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    r.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
    r.z = __builtin_amdgcn_readfirstlane(c < k ? rec : 0);
    r.w = 0x00020000;
    return r;
  };
  const int o0 = (int)(j0 * 4), o1 = (int)(j1 * 4);
  f2v r0[P], r1[P];
#pragma unroll
  for (int q = 0; q < P; ++q) {  // issued before the user staging: independent of it
    const i4v rs = rsrc_of(q);
    r0[q] = rbuf_load_f2(rs, o0, 0, 0);
    r1[q] = rbuf_load_f2(rs, o1, 0, 0);
  }
  for (int t = threadIdx.x; t < UB * kp; t += blockDim.x) {
    const int b = t / kp, c = t % kp;
    const int64_t ur = (b0 + b < n_users) ? user_rows[b0 + b] : -1;
    us[c][b] = (ur >= 0 && c < k) ? U[ur * kp + c] : 0.f;
    if (c == 0) uok[b] = ur >= 0;
  }
  float tb[UB];  // survivor thresholds, read ahead of the loop
#pragma unroll
  for (int b = 0; b < UB; ++b) tb[b] = (FILTER && b0 + b < n_users) ? thr[(int64_t)(b0 + b) * thr_stride] : 0.f;
  __syncthreads();
  f2v acc0[UB], acc1[UB];
#pragma unroll
  for (int b = 0; b < UB; ++b) {
    acc0[b] = f2v{0.f, 0.f};
    acc1[b] = f2v{0.f, 0.f};
  }
  // user values for rank step c + 1 are read from LDS while step c computes
  // (two register sets, alternating with the parity of the unrolled step)
  float4 ub[2][UB / 4];
#pragma unroll
  for (int b = 0; b < UB; b += 4) ub[0][b / 4] = *reinterpret_cast<const float4*>(&us[0][b]);
  for (int c0 = 0; c0 < k; c0 += P) {
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const int c = c0 + q;  // may pass k by < P: zero factors there (us staged 0)
#pragma unroll
      for (int b = 0; b < UB; b += 4) ub[(q + 1) & 1][b / 4] = *reinterpret_cast<const float4*>(&us[c + 1][b]);
      {
        const f2v v0 = r0[q], v1 = r1[q];
#pragma unroll
        for (int b = 0; b < UB; b += 4) {
          const float4 u4 = ub[q & 1][b / 4];
          const float uu[4] = {u4.x, u4.y, u4.z, u4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const f2v us2 = f2v{uu[e], uu[e]};
            const f2v p0 = us2 * v0;
            const f2v p1 = us2 * v1;
            acc0[b + e] = acc0[b + e] + p0;
            acc1[b + e] = acc1[b + e] + p1;
          }
        }
        // refill the slot only once its values are dead, so the load lands in
        // the slot's own registers (no copy waiting on it at the back edge)
        const i4v rs = rsrc_of(c + P);
        r0[q] = rbuf_load_f2(rs, o0, 0, 0);
        r1[q] = rbuf_load_f2(rs, o1, 0, 0);
      }
    }
  }
  if (!FILTER) {
    const float qnan = __builtin_nanf("");
    // pairs (j, j + 1) as one 8-B store when rows are 8-B aligned: a wave
    // then writes 512 contiguous bytes per instruction
    const bool pair = HREC_SCORE_PAIR_STORE && (n_items % 2 == 0) && ((reinterpret_cast<uintptr_t>(out) & 7) == 0);
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      if (b0 + b >= n_users) break;
      float* o = out + (int64_t)(b0 + b) * n_items;
      const bool ok = uok[b];
      if (pair) {
        if (j0 + 1 < n_items) *reinterpret_cast<float2*>(o + j0) = ok ? make_float2(acc0[b].x, acc0[b].y)
                                                                        : make_float2(qnan, qnan);
        if (j1 + 1 < n_items) *reinterpret_cast<float2*>(o + j1) = ok ? make_float2(acc1[b].x, acc1[b].y)
                                                                        : make_float2(qnan, qnan);
        continue;
      }
      if (j0 < n_items) o[j0] = ok ? acc0[b].x : qnan;
      if (j0 + 1 < n_items) o[j0 + 1] = ok ? acc0[b].y : qnan;
      if (j1 < n_items) o[j1] = ok ? acc1[b].x : qnan;
      if (j1 + 1 < n_items) o[j1 + 1] = ok ? acc1[b].y : qnan;
    }
  } else {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      if (b0 + b >= n_users || !uok[b]) continue;  // block-uniform
      const float t = tb[b];
      const float sv[4] = {acc0[b].x, acc0[b].y, acc1[b].x, acc1[b].y};
      const int64_t sj[4] = {j0, j0 + 1, j1, j1 + 1};
      // one compare per user in the common case: nothing of this wave passes
      // (NaN scores fail >= like the per-item test; columns >= n_items may
      // pass here and are dropped by the exact test below)
      const float mx = fmaxf(fmaxf(sv[0], sv[1]), fmaxf(sv[2], sv[3]));
      if (__ballot(mx >= t) == 0) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool pass = sj[e] < n_items && sv[e] >= t;
        const uint64_t m = __ballot(pass);
        if (m == 0) continue;
        int base = 0;
        const int leader = __builtin_ctzll(m);
        if (lane == leader) {
          base = atomicAdd(&cand_n[b0 + b], __popcll(m));
          if (base + __popcll(m) > cap) *overflow = 1;  // this user's survivors exceed the list
        }
        base = __shfl(base, leader, kWave);
        if (pass) {
          const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          if (pos < cap) {
            cand_v[(int64_t)(b0 + b) * cap + pos] = sv[e];
            cand_i[(int64_t)(b0 + b) * cap + pos] = sj[e];
          }
        }
      }
    }
  }
}

// ----------------------------------------------------------------- top-k
// Order: larger value first; equal values -> smaller index first (a stable
// descending sort of the input order). NaN sorts last.
template <typename T>
__device__ __forceinline__ bool better(T va, int64_t ia, T vb, int64_t ib) {
  const bool na = va != va, nb = vb != vb;
  if (na || nb) return !na && nb ? true : (na && nb ? ia < ib : false);
  return va > vb || (va == vb && ia < ib);
}

template <typename T>
struct KV {
  T v;
  int64_t i;
};

template <typename T>
__device__ __forceinline__ KV<T> wave_best(KV<T> x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    KV<T> y;
    y.v = __shfl_xor(x.v, off, kWave);
    y.i = __shfl_xor(x.i, off, kWave);
    // lanes without a candidate carry i = INT64_MAX and lose every comparison
    const bool take = (x.i == INT64_MAX) ? (y.i != INT64_MAX)
                                         : (y.i != INT64_MAX && better(y.v, y.i, x.v, x.i));
    if (take) x = y;
  }
  return x;
}

constexpr int kTopkBlock = 256;
constexpr int kTopkPer = 16;  // elements per thread per segment
constexpr int kTopkSeg = kTopkBlock * kTopkPer;
constexpr int kTopkSelectMax = 1024;  // larger top_k: the sort path (csrc/sort_topk.hip)

// Stage 1: rows x segments; each block selects the top `kk` of its segment
// of one row by kk rounds of block arg-best over elements held in registers.
// `src_idx` (optional) maps positions to original indices (stage 2 input).
template <typename T>
__global__ __launch_bounds__(kTopkBlock) void topk_segment_kernel(const T* __restrict__ vals,
                                                                  const int64_t* __restrict__ src_idx,
                                                                  const int* __restrict__ row_n,
                                                                  int64_t n, int64_t row_stride, int kk,
                                                                  T* __restrict__ out_v,
                                                                  int64_t* __restrict__ out_i,
                                                                  int64_t out_row_stride,
                                                                  const int* __restrict__ gate) {
  __shared__ KV<T> red[kTopkBlock / 64];
  __shared__ int64_t win;
  if (gate && *gate == 0) return;
  const int64_t row = blockIdx.y;
  const int64_t seg0 = (int64_t)blockIdx.x * kTopkSeg;
  const T* __restrict__ rv = vals + row * row_stride;
  const int64_t* __restrict__ ri = src_idx ? src_idx + row * row_stride : nullptr;
  if (row_n) {
    const int64_t rn = row_n[row];
    n = rn < n ? rn : n;
  }
  T v[kTopkPer];
  int64_t id[kTopkPer];
#pragma unroll
  for (int e = 0; e < kTopkPer; ++e) {
    const int64_t p = seg0 + (int64_t)e * kTopkBlock + threadIdx.x;
    if (p < n) {
      v[e] = rv[p];
      id[e] = ri ? ri[p] : p;
    } else {
      v[e] = 0;
      id[e] = -1;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int r = 0; r < kk; ++r) {
    KV<T> best{(T)0, -1};
#pragma unroll
    for (int e = 0; e < kTopkPer; ++e) {
      if (id[e] >= 0 && (best.i < 0 || better(v[e], id[e], best.v, best.i))) best = KV<T>{v[e], id[e]};
    }
    if (best.i < 0) best.i = INT64_MAX;
    KV<T> wb = wave_best(best);
    if (lane == 0) red[w] = wb;
    __syncthreads();
    if (threadIdx.x == 0) {
      KV<T> b = red[0];
      for (int q = 1; q < kTopkBlock / 64; ++q) {
        if (red[q].i == INT64_MAX) continue;
        if (b.i == INT64_MAX || better(red[q].v, red[q].i, b.v, b.i)) b = red[q];
      }
      const int64_t o = row * out_row_stride + (int64_t)blockIdx.x * kk + r;
      out_v[o] = b.v;
      out_i[o] = b.i == INT64_MAX ? -1 : b.i;
      win = b.i;
    }
    __syncthreads();
    const int64_t wi = win;
#pragma unroll
    for (int e = 0; e < kTopkPer; ++e)
      if (id[e] == wi) id[e] = -1;
    __syncthreads();
  }
}

// Small top-k (kk <= 16) of rows of at most kTopkWaveMax elements: one wave
// per row. Each lane streams its elements (p = lane, lane + 64, ...) through a
// sorted register list of its KK best (a compare-exchange chain, no
// branches), then kk rounds of wave arg-best over the list heads, the winner
// popping its head. Same order, same output as topk_segment_kernel, without
// its block barriers.
constexpr int kTopkWaveMax = 8192;

template <typename T, int KK>
__global__ __launch_bounds__(256) void topk_wave_kernel(const T* __restrict__ vals,
                                                        const int64_t* __restrict__ src_idx,
                                                        const int* __restrict__ row_n, int64_t n_rows, int64_t n,
                                                        int64_t row_stride, int kk, T* __restrict__ out_v,
                                                        int64_t* __restrict__ out_i, int64_t out_row_stride,
                                                        const int* __restrict__ gate) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n_rows || (gate && *gate == 0)) return;  // wave-uniform
  if (row_n) {
    const int64_t rn = row_n[row];
    n = rn < n ? rn : n;
  }
  const T* __restrict__ rv = vals + row * row_stride;
  const int64_t* __restrict__ ri = src_idx ? src_idx + row * row_stride : nullptr;
  T lv[KK];
  int64_t li[KK];
#pragma unroll
  for (int j = 0; j < KK; ++j) {
    lv[j] = (T)0;
    li[j] = INT64_MAX;  // empty slot: loses to every element
  }
  constexpr int B = 8;  // loads in flight per lane before the first insertion
  for (int64_t p0 = lane; p0 < n; p0 += 64 * B) {
    T bv[B];
    int64_t bi[B];
#pragma unroll
    for (int e = 0; e < B; ++e) {
      const int64_t p = p0 + 64 * e;
      const bool in = p < n;
      bv[e] = in ? rv[p] : (T)0;
      bi[e] = in ? (ri ? ri[p] : p) : -1;
    }
#pragma unroll
    for (int e = 0; e < B; ++e) {
      T xv = bv[e];
      int64_t xi = bi[e] < 0 ? INT64_MAX : bi[e];  // absent: an empty slot, inserts as a no-op
#pragma unroll
      for (int j = 0; j < KK; ++j) {
        const bool sw = xi != INT64_MAX && (li[j] == INT64_MAX || better(xv, xi, lv[j], li[j]));
        const T tv = lv[j];
        const int64_t ti = li[j];
        lv[j] = sw ? xv : tv;
        li[j] = sw ? xi : ti;
        xv = sw ? tv : xv;
        xi = sw ? ti : xi;
      }
    }
  }
  for (int r = 0; r < kk; ++r) {
    const KV<T> w = wave_best(KV<T>{lv[0], li[0]});
    if (lane == 0) {
      const int64_t o = row * out_row_stride + r;
      out_v[o] = w.i == INT64_MAX ? (T)0 : w.v;
      out_i[o] = w.i == INT64_MAX ? -1 : w.i;
    }
    if (w.i != INT64_MAX && li[0] == w.i) {  // the (unique) owner pops its head
#pragma unroll
      for (int j = 0; j + 1 < KK; ++j) {
        lv[j] = lv[j + 1];
        li[j] = li[j + 1];
      }
      li[KK - 1] = INT64_MAX;
    }
  }
}

// Survivor threshold from a sample row (one wave per row, kk <= 64): the
// kk-th largest of the 64 lane maxima (lane l: elements l, l + 64, ...). Those
// are kk distinct sample elements, so the value bounds the row's kk-th best
// from below, which is all the filter needs (the final top-k is exact). NaN
// elements are ignored (fmaxf); a row without a number yields -inf.
__global__ __launch_bounds__(256) void sample_threshold_kernel(const float* __restrict__ vals, int64_t n_rows,
                                                               int64_t n, int kk, float* __restrict__ thr,
                                                               int* __restrict__ zero_cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n_rows) return;  // wave-uniform
  const float* __restrict__ rv = vals + row * n;
  float m = -__builtin_inff();
  int64_t p = lane;
  for (; p + 64 * 3 < n; p += 64 * 4) {  // four loads in flight per lane
    const float a = rv[p], b = rv[p + 64], c = rv[p + 128], d = rv[p + 192];
    m = fmaxf(m, fmaxf(fmaxf(a, b), fmaxf(c, d)));
  }
  for (; p < n; p += 64) m = fmaxf(m, rv[p]);
  float t = -__builtin_inff();
  for (int r = 0; r < kk; ++r) {
    float w = m;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) w = fmaxf(w, __shfl_xor(w, off, kWave));
    t = w;
    // retire one lane holding the maximum (the lowest such lane)
    const uint64_t hold = __ballot(m == w);
    if (hold && lane == __builtin_ctzll(hold)) m = -__builtin_inff();
  }
  if (lane == 0) {
    thr[row] = t;
    if (zero_cnt) zero_cnt[row] = 0;
  }
}

// ---------------------------------------------------------------- fusion
// sklearn MinMaxScaler.fit_transform (container sklearn _data.py:518-522,
// 261-262): scale = 1/range (range < 10*eps -> 1), min_ = 0 - min*scale,
// y = x*scale + min_ ; two roundings each, in the input dtype.
__global__ __launch_bounds__(256) void minmax_partial_kernel(const double* __restrict__ als,
                                                             const void* __restrict__ tt, int tt_f32,
                                                             int64_t n, double* __restrict__ part) {
  __shared__ double sh[4][256];
  double amin = DBL_MAX, amax = -DBL_MAX, tmin = DBL_MAX, tmax = -DBL_MAX;
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (int64_t)gridDim.x * 256) {
    const double a = als[p];
    const double t = tt_f32 ? (double)((const float*)tt)[p] : ((const double*)tt)[p];
    amin = fmin(amin, a);
    amax = fmax(amax, a);
    tmin = fmin(tmin, t);
    tmax = fmax(tmax, t);
  }
  sh[0][threadIdx.x] = amin;
  sh[1][threadIdx.x] = amax;
  sh[2][threadIdx.x] = tmin;
  sh[3][threadIdx.x] = tmax;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      sh[0][threadIdx.x] = fmin(sh[0][threadIdx.x], sh[0][threadIdx.x + s]);
      sh[1][threadIdx.x] = fmax(sh[1][threadIdx.x], sh[1][threadIdx.x + s]);
      sh[2][threadIdx.x] = fmin(sh[2][threadIdx.x], sh[2][threadIdx.x + s]);
      sh[3][threadIdx.x] = fmax(sh[3][threadIdx.x], sh[3][threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x < 4) part[blockIdx.x * 4 + threadIdx.x] = sh[threadIdx.x][0];
}

// coef = {als_scale, als_min_, tt_scale, tt_min_} as doubles (the tt pair is
// the exact f32 values widened when tt_f32).
__global__ void minmax_final_kernel(const double* __restrict__ part, int nparts, int tt_f32,
                                    double* __restrict__ coef, double* __restrict__ out_minmax) {
  if (threadIdx.x != 0) return;
  double amin = DBL_MAX, amax = -DBL_MAX, tmin = DBL_MAX, tmax = -DBL_MAX;
  for (int q = 0; q < nparts; ++q) {
    amin = fmin(amin, part[4 * q + 0]);
    amax = fmax(amax, part[4 * q + 1]);
    tmin = fmin(tmin, part[4 * q + 2]);
    tmax = fmax(tmax, part[4 * q + 3]);
  }
  if (out_minmax) {  // the fitted MinMaxScalers' data_min_ / data_max_ (src/hybrid_system.py:66-67)
    out_minmax[0] = amin;
    out_minmax[1] = amax;
    out_minmax[2] = tmin;
    out_minmax[3] = tmax;
  }
  double arange = amax - amin;
  if (arange < 10.0 * DBL_EPSILON) arange = 1.0;
  const double ascale = 1.0 / arange;
  coef[0] = ascale;
  coef[1] = 0.0 - amin * ascale;
  if (tt_f32) {
    const float fmin_ = (float)tmin, fmax_ = (float)tmax;
    float frange = fmax_ - fmin_;
    if (frange < 10.0f * FLT_EPSILON) frange = 1.0f;
    const float fscale = 1.0f / frange;
    const float fmin2 = 0.0f - fmin_ * fscale;
    coef[2] = (double)fscale;
    coef[3] = (double)fmin2;
  } else {
    double trange = tmax - tmin;
    if (trange < 10.0 * DBL_EPSILON) trange = 1.0;
    const double tscale = 1.0 / trange;
    coef[2] = tscale;
    coef[3] = 0.0 - tmin * tscale;
  }
}

// fused = w0*als_norm + w1*tt_norm, f64 (numpy 1.21 scalar promotion: the
// f32 tt_norm element is widened before the multiply — SURVEY App. A.3).
__global__ __launch_bounds__(256) void fuse_kernel(const double* __restrict__ als, const void* __restrict__ tt,
                                                   int tt_f32, int64_t n, const double* __restrict__ coef,
                                                   double w0, double w1, double* __restrict__ fused) {
#pragma clang fp contract(off)
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  const double an = als[p] * coef[0] + coef[1];
  double tn;
  if (tt_f32) {
    const float x = ((const float*)tt)[p];
    const float y = x * (float)coef[2] + (float)coef[3];
    tn = (double)y;
  } else {
    tn = ((const double*)tt)[p] * coef[2] + coef[3];
  }
  fused[p] = w0 * an + w1 * tn;
}


// ------------------------------------------------------- cold-start cosine
// ALSModel._find_similar_items (src/als_model.py:93-104): sklearn
// cosine_similarity([target], [other]) = dot(a/|a|, b/|b|) with a zero norm
// replaced by 1. One thread per (query, item); the query's own row -> -inf so
// it never ranks (the reference skips it).
__global__ __launch_bounds__(256) void cosine_kernel(const double* __restrict__ feats, int64_t n_items, int dim,
                                                     const int64_t* __restrict__ qrows, double* __restrict__ out) {
#pragma clang fp contract(off)
  const int64_t q = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n_items) return;
  const int64_t qr = qrows[q];
  double* o = out + q * n_items;
  if (j == qr) {
    o[j] = -__builtin_inf();
    return;
  }
  const double* a = feats + qr * dim;
  const double* b = feats + j * dim;
  double na = 0.0, nb = 0.0;
  for (int c = 0; c < dim; ++c) {
    na = na + a[c] * a[c];
    nb = nb + b[c] * b[c];
  }
  na = sqrt(na);
  nb = sqrt(nb);
  if (na == 0.0) na = 1.0;
  if (nb == 0.0) nb = 1.0;
  double dot = 0.0;
  for (int c = 0; c < dim; ++c) dot = dot + (a[c] / na) * (b[c] / nb);
  o[j] = dot;
}


// --------------------------------------------- batched fusion (K9, rows)
// Per-row min / max of an f32 score matrix (NaN ignored, like np.nanmin):
// out[r] = min, out[n_rows + r] = max (two contiguous halves, so the
// cross-shard reduction is one MIN and one MAX all-reduce). One block per row.
// Per-row min / max (NaN ignored, like fminf). One 1024-thread block per
// row streams it with 16-B loads (rows 16-B aligned) — HBM-bound.
__global__ __launch_bounds__(1024) void rows_minmax_kernel(const float* __restrict__ x, int64_t n, int64_t ld,
                                                           int vec4, float* __restrict__ out) {
  __shared__ float smin[16], smax[16];
  const float* r = x + (int64_t)blockIdx.x * ld;
  float lo = __builtin_inff(), hi = -__builtin_inff();
  int64_t j0 = 0;
  if (vec4) {
    const int64_t n4 = n >> 2;
    const float4* r4 = reinterpret_cast<const float4*>(r);
    for (int64_t j = threadIdx.x; j < n4; j += 1024) {
      const float4 v = r4[j];
      lo = fminf(fminf(lo, v.x), fminf(v.y, fminf(v.z, v.w)));
      hi = fmaxf(fmaxf(hi, v.x), fmaxf(v.y, fmaxf(v.z, v.w)));
    }
    j0 = n4 << 2;
  }
  for (int64_t j = j0 + threadIdx.x; j < n; j += 1024) {
    lo = fminf(lo, r[j]);
    hi = fmaxf(hi, r[j]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, off, kWave));
    hi = fmaxf(hi, __shfl_xor(hi, off, kWave));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smin[w] = lo;
    smax[w] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < 16; ++q) {
      lo = fminf(lo, smin[q]);
      hi = fmaxf(hi, smax[q]);
    }
    out[blockIdx.x] = lo;              // mins  [n_rows]
    out[gridDim.x + blockIdx.x] = hi;  // maxes [n_rows]
  }
}

// fused[r][j] = w0 * minmax64(als[r][j]) + w1 * (double)minmax32(tt[r][j]),
// with each row's min/max given (global over every shard of the row): the
// ALS side is min-max scaled in f64 (the reference's als scores are Python
// floats), the two-tower side in f32 (np.float32 scores), then f64 fusion
// with numpy 1.21's scalar promotion — hrec_fuse_topk per row.
__global__ __launch_bounds__(256) void fuse_rows_kernel(const float* __restrict__ als, const float* __restrict__ tt,
                                                        int64_t n, int64_t ld, const float* __restrict__ als_mm,
                                                        const float* __restrict__ tt_mm, double w0, double w1,
                                                        double* __restrict__ fused) {
#pragma clang fp contract(off)
  const int64_t r = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const int64_t R = gridDim.y;  // min/max layout: [2][n_rows]
  const double amin = (double)als_mm[r], amax = (double)als_mm[R + r];
  double arange = amax - amin;
  if (arange < 10.0 * DBL_EPSILON) arange = 1.0;
  const double ascale = 1.0 / arange;
  const double amin_ = 0.0 - amin * ascale;
  const float tmin = tt_mm[r], tmax = tt_mm[R + r];
  float trange = tmax - tmin;
  if (trange < 10.0f * FLT_EPSILON) trange = 1.0f;
  const float tscale = 1.0f / trange;
  const float tmin_ = 0.0f - tmin * tscale;
  const double an = (double)als[r * ld + j] * ascale + amin_;
  const float tn = tt[r * ld + j] * tscale + tmin_;
  fused[r * n + j] = w0 * an + w1 * (double)tn;
}

// fuse_rows_kernel's arithmetic + a stable top-kk (kk <= kFuseK) of each
// segment of kFuseSeg items, without materialising the fused row. One WAVE
// per segment (no block barriers). Each fused f64 becomes an order-preserving
// u64 key (NaN lowest, as `better` ranks it), so every comparison is one
// integer compare; lane l holds items seg0 + 64 e + l (ascending e =
// ascending index, so a strict '>' keeps the earlier item on ties).
//   1. t = the kk-th best of the 64 lane maxima (kk rounds of a wave
//      arg-best; the winning LANE drops out) — a lower bound of the
//      segment's kk-th best, since those kk maxima are kk distinct items;
//   2. items not worse than t are the candidates (ballot-compacted into LDS;
//      typically ~kk of them; more than 64 — heavy ties — falls back to
//      exact rescans);
//   3. kk rounds of a wave arg-best over the candidates (key desc, index asc)
//      -> [row][seg*kk] (value, index).
constexpr int kFuseK = 8;
#ifndef HREC_FUSE_PER
#define HREC_FUSE_PER 16
#endif
constexpr int kFusePer = HREC_FUSE_PER;  // items per lane per segment
constexpr int kFuseSeg = 64 * kFusePer;
#ifndef HREC_FUSE_RANK
#define HREC_FUSE_RANK 1  // selections by rank among <= 64 entries (LDS broadcast reads) instead of arg-best rounds
#endif
constexpr bool kFuseRank = HREC_FUSE_RANK;

__device__ __forceinline__ uint64_t order_key(double v) {
  if (v != v) return 0;  // NaN ranks below every number
  const uint64_t b = (uint64_t)__double_as_longlong(v + 0.0);  // -0 -> +0 (they compare equal)
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double key_value(uint64_t k) {
  if (k == 0) return __builtin_nan("");
  return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k));
}

struct KI {
  uint64_t k;
  int64_t i;  // INT64_MAX: no item
};
__device__ __forceinline__ bool ki_better(const KI& a, const KI& b) {  // a ranks before b
  return a.i != INT64_MAX && (b.i == INT64_MAX || a.k > b.k || (a.k == b.k && a.i < b.i));
}
__device__ __forceinline__ KI wave_best_ki(KI x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    KI y;
    y.k = ((uint64_t)(uint32_t)__shfl_xor((int)(x.k >> 32), off, kWave) << 32) |
          (uint32_t)__shfl_xor((int)x.k, off, kWave);
    y.i = __shfl_xor(x.i, off, kWave);
    if (ki_better(y, x)) x = y;
  }
  return x;
}

// One segment (seg of row r, R rows) on one wave; ck / ce: the wave's 128
// LDS slots ([64, 128): scratch of non-candidates).
template <int KK>
__device__ __forceinline__ void fuse_segment_one(
    int64_t seg, int64_t r, int64_t R, const float* __restrict__ als, const float* __restrict__ tt, int64_t n,
    int64_t ld, int64_t segs, const float* __restrict__ als_mm, const float* __restrict__ tt_mm, double w0, double w1,
    double* __restrict__ cand_v, int64_t* __restrict__ cand_i, uint64_t* __restrict__ ck, int* __restrict__ ce) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const double amin = (double)als_mm[r], amax = (double)als_mm[R + r];
  double arange = amax - amin;
  if (arange < 10.0 * DBL_EPSILON) arange = 1.0;
  const double ascale = 1.0 / arange;
  const double amin_ = 0.0 - amin * ascale;
  const float tmin = tt_mm[r], tmax = tt_mm[R + r];
  float trange = tmax - tmin;
  if (trange < 10.0f * FLT_EPSILON) trange = 1.0f;
  const float tscale = 1.0f / trange;
  const float tmin_ = 0.0f - tmin * tscale;
  const int64_t seg0 = seg * kFuseSeg;
  const float* __restrict__ ar = als + r * ld + seg0 + lane;
  const float* __restrict__ tr = tt + r * ld + seg0 + lane;
  const int nvalid = (int)((n - seg0) < kFuseSeg ? (n - seg0) : kFuseSeg);  // items of this segment
  uint64_t key[kFusePer];
  float av[kFusePer], tv[kFusePer];
  if (nvalid == kFuseSeg) {  // full segment: unconditional loads
#pragma unroll
    for (int e = 0; e < kFusePer; ++e) {
      av[e] = ar[e * 64];
      tv[e] = tr[e * 64];
    }
  } else {
#pragma unroll
    for (int e = 0; e < kFusePer; ++e) {
      const int off = e * 64 + lane < nvalid ? e * 64 : 0;  // the lane's first item is in range
      av[e] = ar[off];
      tv[e] = tr[off];
    }
  }
#pragma unroll
  for (int e = 0; e < kFusePer; ++e) {
    const double an = (double)av[e] * ascale + amin_;
    const float tn = tv[e] * tscale + tmin_;
    const uint64_t kv = order_key(w0 * an + w1 * (double)tn);
    key[e] = e * 64 + lane < nvalid ? kv : 0;
  }
  const int nmine = nvalid > lane ? (nvalid - lane + 63) >> 6 : 0;  // live items of this lane
  // 1. lane arg-best (strict '>' in ascending e keeps the earliest of equals)
  uint64_t bk = key[0];
  int be = 0;
#pragma unroll
  for (int e = 1; e < kFusePer; ++e) {
    const bool gt = key[e] > bk;
    bk = gt ? key[e] : bk;
    be = gt ? e : be;
  }
  KI mine{bk, nmine > 0 ? seg0 + (int64_t)be * 64 + lane : INT64_MAX};
  KI t{0, INT64_MAX};
  if constexpr (kFuseRank) {
    // t = the min(kk, live lanes)-th best lane maximum, by each lane's RANK
    // among the 64 maxima (one pass of broadcast LDS reads, no dependent
    // cross-lane rounds); in-segment positions order equal keys
    const int mpos = nmine > 0 ? be * 64 + lane : -1;
    ck[64 + lane] = bk;
    ce[64 + lane] = mpos;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int rank = 0;
#pragma unroll 8
    for (int q = 0; q < 64; ++q) {
      const uint64_t ok = ck[64 + q];
      const int op = ce[64 + q];
      rank += (op >= 0 && (mpos < 0 || ok > bk || (ok == bk && op < mpos))) ? 1 : 0;
    }
    const int nvl = __popcll(__ballot(mpos >= 0));
    const int target = (nvl < KK ? nvl : KK) - 1;
    const uint64_t hit = __ballot(mpos >= 0 && rank == target);
    if (hit) {
      const int src = __builtin_ctzll(hit);
      t.k = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(bk >> 32), src) << 32) |
            (uint32_t)__builtin_amdgcn_readlane((int)bk, src);
      t.i = seg0 + __builtin_amdgcn_readlane(mpos, src);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    for (int q = 0; q < KK; ++q) {
      const KI w = wave_best_ki(mine);
      if (w.i == INT64_MAX) break;
      t = w;
      if (w.i == mine.i) mine.i = INT64_MAX;
    }
  }
  // 2. candidates: items not worse than t (no t: fewer than kk items, take all)
  int nc = 0;
  bool overflow = false;
#pragma unroll
  for (int e = 0; e < kFusePer; ++e) {
    const int64_t j = seg0 + (int64_t)e * 64 + lane;
    const bool live = e < nmine;
    const bool c = live && (t.i == INT64_MAX || key[e] > t.k || (key[e] == t.k && j <= t.i));
    const uint64_t m = __ballot(c);
    const int cnt = __popcll(m);
    if (nc + cnt > 64) {
      overflow = true;
      break;
    }
    const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const int slot = c ? nc + below : 64 + lane;  // branch-free append
    ck[slot] = key[e];
    ce[slot] = e * 64 + lane;
    nc += cnt;
  }
  const int64_t obase = r * segs * KK + seg * KK;
  if (!overflow) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if constexpr (kFuseRank) {
      // each candidate's rank among the nc candidates = its output slot
      const uint64_t mk = lane < nc ? ck[lane] : 0;
      const int mp = lane < nc ? ce[lane] : 0;
      int rank = 0;
      for (int q = 0; q < nc; ++q) {
        const uint64_t ok = ck[q];
        const int op = ce[q];
        rank += (ok > mk || (ok == mk && op < mp)) ? 1 : 0;
      }
      if (lane < nc && rank < KK) {
        cand_v[obase + rank] = key_value(mk);
        cand_i[obase + rank] = seg0 + mp;
      }
      if (lane >= nc && lane < KK) {  // fewer candidates than kk: empty slots
        cand_v[obase + lane] = key_value(0);
        cand_i[obase + lane] = -1;
      }
      return;
    }
    KI c{0, INT64_MAX};
    if (lane < nc) c = KI{ck[lane], seg0 + ce[lane]};
    for (int q = 0; q < KK; ++q) {
      const KI w = wave_best_ki(c);
      if (lane == 0) {
        cand_v[obase + q] = key_value(w.k);
        cand_i[obase + q] = w.i == INT64_MAX ? -1 : w.i;
      }
      if (w.i == c.i) c.i = INT64_MAX;
    }
    return;
  }
  // heavy ties: exact selection by rescans (the winning lane drops its item)
  uint32_t live_mask = nmine >= 32 ? 0xffffffffu : ((1u << nmine) - 1u);  // kFusePer <= 32
  auto rescan = [&](KI& m2) {
    m2 = KI{0, INT64_MAX};
#pragma unroll
    for (int e = 0; e < kFusePer; ++e) {
      const KI x{key[e], seg0 + (int64_t)e * 64 + lane};
      if (((live_mask >> e) & 1u) && ki_better(x, m2)) m2 = x;
    }
  };
  KI m2;
  rescan(m2);
  for (int q = 0; q < KK; ++q) {
    const KI w = wave_best_ki(m2);
    if (lane == 0) {
      cand_v[obase + q] = key_value(w.k);
      cand_i[obase + q] = w.i == INT64_MAX ? -1 : w.i;
    }
    if (w.i != INT64_MAX && w.i == m2.i) {
      live_mask &= ~(1u << (int)((w.i - seg0) >> 6));
      rescan(m2);
    }
  }
}

template <int KK>
__global__ __launch_bounds__(256) void fuse_segment_topk_kernel(
    const float* __restrict__ als, const float* __restrict__ tt, int64_t n, int64_t ld, int64_t segs,
    const float* __restrict__ als_mm, const float* __restrict__ tt_mm, double w0, double w1,
    double* __restrict__ cand_v, int64_t* __restrict__ cand_i, const int* __restrict__ gate, int* __restrict__ clear) {
  // clear (the sample launch): reset the filter's overflow flag for this call
  if (clear && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *clear = 0;
  if (gate && *gate == 0) return;
  __shared__ uint64_t ck_sh[4][128];
  __shared__ int ce_sh[4][128];
  const int wv = threadIdx.x >> 6;
  // block-stride over the row's segment groups (a gated launch uses one block
  // per row, so skipping it costs a small grid)
  for (int64_t sb = blockIdx.x; sb * 4 < segs; sb += gridDim.x) {
    const int64_t seg = sb * 4 + wv;
    if (seg < segs)
      fuse_segment_one<KK>(seg, blockIdx.y, gridDim.y, als, tt, n, ld, segs, als_mm, tt_mm, w0, w1, cand_v, cand_i,
                           ck_sh[wv], ce_sh[wv]);
  }
}

// Threshold filter for the batched fusion top-k (kk <= kFuseK): the same
// fused f64 keys as fuse_segment_topk_kernel, one wave per segment, but each
// row first takes a threshold key tk = the best of its sample segments'
// kk-th best keys (fuse_segment_topk_kernel over the row's first G segments
// -> samp). Those are kk distinct items of the row, so at least kk items have
// key >= tk and the row's top kk all do. Per item: the fusion, one compare
// and a ballot; the (few) items with key >= tk are compacted into LDS and
// the segment's stable top-kk among them is taken by rank (each candidate
// counts the better ones, a handful of broadcast LDS reads) -> [row][seg*kk]
// like fuse_segment_topk_kernel, and the same merge follows. A segment with
// more than kFuseSlots candidates (heavy ties, or a row whose best items
// cluster) raises *overflow, which gates the exact segment path on the
// device (the sample launch of fuse_segment_topk_kernel resets it first).
constexpr int kFuseSlots = 64;
__global__ __launch_bounds__(256) void fuse_filter_kernel(
    const float* __restrict__ als, const float* __restrict__ tt, int64_t n, int64_t ld, int64_t segs,
    const float* __restrict__ als_mm, const float* __restrict__ tt_mm, double w0, double w1,
    const double* __restrict__ samp, int G, int kk, double* __restrict__ cand_v, int64_t* __restrict__ cand_i,
    int* __restrict__ overflow) {
#pragma clang fp contract(off)
  __shared__ uint64_t ck_sh[4][kFuseSlots];
  __shared__ int ce_sh[4][kFuseSlots];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t seg = (int64_t)blockIdx.x * 4 + wv;
  if (seg >= segs) return;
  const int64_t r = blockIdx.y;
  const int64_t R = gridDim.y;
  uint64_t tk = 0;
  for (int g = 0; g < G; ++g) {
    const uint64_t k = order_key(samp[(r * G + g) * kk + kk - 1]);
    tk = k > tk ? k : tk;
  }
  const double amin = (double)als_mm[r], amax = (double)als_mm[R + r];
  double arange = amax - amin;
  if (arange < 10.0 * DBL_EPSILON) arange = 1.0;
  const double ascale = 1.0 / arange;
  const double amin_ = 0.0 - amin * ascale;
  const float tmin = tt_mm[r], tmax = tt_mm[R + r];
  float trange = tmax - tmin;
  if (trange < 10.0f * FLT_EPSILON) trange = 1.0f;
  const float tscale = 1.0f / trange;
  const float tmin_ = 0.0f - tmin * tscale;
  const int64_t seg0 = seg * kFuseSeg;
  const float* __restrict__ ar = als + r * ld + seg0 + lane;
  const float* __restrict__ tr = tt + r * ld + seg0 + lane;
  const int nvalid = (int)((n - seg0) < kFuseSeg ? (n - seg0) : kFuseSeg);
  float av[kFusePer], tv[kFusePer];
  if (nvalid == kFuseSeg) {
#pragma unroll
    for (int e = 0; e < kFusePer; ++e) {
      av[e] = ar[e * 64];
      tv[e] = tr[e * 64];
    }
  } else {
#pragma unroll
    for (int e = 0; e < kFusePer; ++e) {
      const int off = e * 64 + lane < nvalid ? e * 64 : 0;
      av[e] = ar[off];
      tv[e] = tr[off];
    }
  }
  int nc = 0;
#pragma unroll
  for (int e = 0; e < kFusePer; ++e) {
    const double an = (double)av[e] * ascale + amin_;
    const float tn = tv[e] * tscale + tmin_;
    const uint64_t key = order_key(w0 * an + w1 * (double)tn);
    const bool c = e * 64 + lane < nvalid && key >= tk;
    const uint64_t m = __ballot(c);
    if (m == 0) continue;  // wave-uniform
    const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const int slot = nc + below;
    if (c && slot < kFuseSlots) {
      ck_sh[wv][slot] = key;
      ce_sh[wv][slot] = e * 64 + lane;
    }
    nc += __popcll(m);
  }
  if (nc > kFuseSlots) {
    if (lane == 0) *overflow = 1;
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // each candidate's rank among the nc (key desc, position asc) = its slot
  const uint64_t mk = lane < nc ? ck_sh[wv][lane] : 0;
  const int mp = lane < nc ? ce_sh[wv][lane] : 0;
  int rank = 0;
  for (int q = 0; q < nc; ++q) {
    const uint64_t ok = ck_sh[wv][q];
    const int op = ce_sh[wv][q];
    rank += (ok > mk || (ok == mk && op < mp)) ? 1 : 0;
  }
  const int64_t obase = (r * segs + seg) * kk;
  if (lane < nc && rank < kk) {
    cand_v[obase + rank] = key_value(mk);
    cand_i[obase + rank] = seg0 + mp;
  }
  if (lane >= nc && lane < kk) {  // fewer candidates than kk: empty slots
    cand_v[obase + lane] = key_value(0);
    cand_i[obase + lane] = -1;
  }
}

__global__ void add_offset_kernel(int64_t* __restrict__ idx, int64_t n, int64_t off) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n && idx[i] >= 0) idx[i] += off;
}

}  // namespace hrec

using namespace hrec;

// Workspace for a stable top-k of n_rows rows of n elements (bytes) by the
// segment selections (kk <= kTopkSelectMax). Each pass keeps kk of every
// kTopkSeg elements, so it shrinks the row only while kk < kTopkSeg / 2; the
// loop stops as soon as a pass would not shrink it (larger kk go through the
// sort path, csrc/sort_topk.hip).
namespace hrec {
size_t topk_ws_bytes(int64_t n_rows, int64_t n, int kk, size_t elem) {
  size_t total = 0;
  int64_t m = n;
  if (kk < 1 || kk > kTopkSelectMax) return 256;
  while (true) {
    const int64_t segs = (m + kTopkSeg - 1) / kTopkSeg;
    if (segs <= 1) break;
    const int64_t cand = segs * kk;
    if (cand >= m) break;
    total += (size_t)n_rows * (size_t)cand * (elem + 8);
    m = cand;
  }
  return total + 256;
}
}  // namespace hrec

namespace hrec {
template <typename T>
int topk_rows(const T* vals, int64_t n_rows, int64_t n, int64_t row_stride, int kk, int64_t* out_idx,
              T* out_val, void* ws, size_t ws_bytes, hipStream_t s, const int64_t* src_idx, const int* row_n,
              const int* gate) {
  // Multi-pass: segments -> candidates (kk per segment) -> ... -> one segment.
  const T* cur_v = vals;
  const int64_t* cur_i = src_idx;
  int64_t m = n, stride = row_stride;
  char* w = (char*)ws;
  size_t used = 0;
  while (true) {
    const int64_t segs = (m + kTopkSeg - 1) / kTopkSeg;
    if (segs <= 1 || (m <= kTopkWaveMax && kk <= 16)) {
      if (kk <= 16 && m <= kTopkWaveMax) {
        const dim3 g((unsigned)((n_rows + 3) / 4));
#define HREC_TOPK_WAVE(KK)                                                                                    \
  hipLaunchKernelGGL((topk_wave_kernel<T, KK>), g, dim3(256), 0, s, cur_v, cur_i, row_n, n_rows, m, stride, kk, \
                     out_val, out_idx, (int64_t)kk, gate)
        if (kk <= 2)
          HREC_TOPK_WAVE(2);
        else if (kk <= 4)
          HREC_TOPK_WAVE(4);
        else if (kk == 5)  // the reference's default top_k: 5-deep lane lists
          HREC_TOPK_WAVE(5);
        else if (kk <= 8)
          HREC_TOPK_WAVE(8);
        else
          HREC_TOPK_WAVE(16);
#undef HREC_TOPK_WAVE
        return check_launch("topk_wave_kernel");
      }
      hipLaunchKernelGGL((topk_segment_kernel<T>), dim3(1, (unsigned)n_rows), dim3(kTopkBlock), 0, s, cur_v,
                         cur_i, row_n, m, stride, kk, out_val, out_idx, (int64_t)kk, gate);
      return check_launch("topk_segment_kernel");
    }
    const int64_t cand = segs * kk;
    const size_t vb = (size_t)n_rows * cand * sizeof(T), ib = (size_t)n_rows * cand * 8;
    if (used + vb + ib > ws_bytes) {
      set_error("topk: workspace too small");
      return HREC_E_INVALID;
    }
    int64_t* ni = (int64_t*)(w + used);
    T* nv = (T*)(w + used + ib);
    used += vb + ib;
    hipLaunchKernelGGL((topk_segment_kernel<T>), dim3((unsigned)segs, (unsigned)n_rows), dim3(kTopkBlock), 0, s,
                       cur_v, cur_i, row_n, m, stride, kk, nv, ni, cand, gate);
    int rc = check_launch("topk_segment_kernel");
    if (rc) return rc;
    cur_v = nv;
    cur_i = ni;
    row_n = nullptr;  // later passes: every row holds segs * kk entries
    m = cand;
    stride = cand;
  }
}
template int topk_rows<float>(const float*, int64_t, int64_t, int64_t, int, int64_t*, float*, void*, size_t,
                              hipStream_t, const int64_t*, const int*, const int*);
template int topk_rows<double>(const double*, int64_t, int64_t, int64_t, int, int64_t*, double*, void*, size_t,
                               hipStream_t, const int64_t*, const int*, const int*);
}  // namespace hrec

extern "C" int hrec_als_score(const float* user_factors, const int64_t* user_rows, int n_users,
                              const float* item_factors_t, int64_t ld_items, const int64_t* item_rows,
                              int64_t n_items, int k, int kp, float* out, void* stream) {
  HREC_REQUIRE(hrec_factor_ld_ok(kp), "als_score: kp must be 16, 32, 64, 96, 128, 192 or 256");
  HREC_REQUIRE(k >= 1 && k <= kp, "als_score: need 1 <= k <= kp");
  HREC_REQUIRE(n_users >= 0 && n_items >= 0 && ld_items >= 0, "als_score: negative size");
  if (n_users == 0 || n_items == 0) return HREC_OK;
  HREC_REQUIRE(user_factors && user_rows && item_factors_t && out, "als_score: null pointer");
  HREC_REQUIRE(item_rows != nullptr || n_items <= ld_items, "als_score: n_items > ld_items");
  constexpr int UB = 16;
  if (item_rows == nullptr && ld_items % 2 == 0 && ld_items < ((int64_t)1 << 29) &&
      (reinterpret_cast<uintptr_t>(item_factors_t) & 7) == 0) {
    // every item in order: the packed-f32 kernel (same JVM-exact chain)
    const dim3 grid((unsigned)((n_users + UB - 1) / UB), (unsigned)((n_items + 1023) / 1024));
    hipLaunchKernelGGL((als_score_fast_kernel<UB, false>), grid, dim3(256), 0, as_stream(stream), user_factors,
                       user_rows, n_users, item_factors_t, ld_items, n_items, k, kp, out, nullptr, 0, 0, nullptr,
                       nullptr, nullptr, nullptr);
    return check_launch("als_score_fast_kernel");
  }
  const dim3 grid((unsigned)((n_items + 255) / 256), (unsigned)((n_users + UB - 1) / UB));
  hipLaunchKernelGGL((als_score_kernel<UB>), grid, dim3(256), 0, as_stream(stream), user_factors, user_rows,
                     n_users, item_factors_t, ld_items, item_rows, n_items, k, kp, out);
  return check_launch("als_score_kernel");
}

extern "C" size_t hrec_topk_workspace_bytes(int64_t n_rows, int64_t n, int top_k, int is_f64) {
  const int64_t kk = top_k < n ? top_k : n;
  if (kk > kTopkSelectMax) return sort_topk_ws_bytes(n_rows, n);
  return topk_ws_bytes(n_rows, n, (int)kk, is_f64 ? 8 : 4);
}

extern "C" int hrec_topk_f32(const float* vals, int64_t n_rows, int64_t n, int64_t row_stride, int top_k,
                             int64_t* out_idx, float* out_val, void* workspace, size_t workspace_bytes,
                             void* stream) {
  HREC_REQUIRE(n_rows >= 0 && n >= 0 && row_stride >= n, "topk_f32: bad shape");
  HREC_REQUIRE(top_k >= 1, "topk_f32: top_k must be >= 1");
  if (n_rows == 0 || n == 0) return HREC_OK;
  HREC_REQUIRE(n_rows < 65536, "topk_f32: at most 65535 rows per call");
  HREC_REQUIRE(vals && out_idx && out_val, "topk_f32: null pointer");
  const int kk = (int)(top_k < n ? top_k : n);
  if (kk > kTopkSelectMax)
    return sort_topk_rows<float>(vals, n_rows, n, row_stride, kk, out_idx, out_val, workspace, workspace_bytes,
                                as_stream(stream));
  return topk_rows<float>(vals, n_rows, n, row_stride, kk, out_idx, out_val, workspace, workspace_bytes,
                          as_stream(stream));
}

extern "C" int hrec_topk_f64(const double* vals, int64_t n_rows, int64_t n, int64_t row_stride, int top_k,
                             int64_t* out_idx, double* out_val, void* workspace, size_t workspace_bytes,
                             void* stream) {
  HREC_REQUIRE(n_rows >= 0 && n >= 0 && row_stride >= n, "topk_f64: bad shape");
  HREC_REQUIRE(top_k >= 1, "topk_f64: top_k must be >= 1");
  if (n_rows == 0 || n == 0) return HREC_OK;
  HREC_REQUIRE(n_rows < 65536, "topk_f64: at most 65535 rows per call");
  HREC_REQUIRE(vals && out_idx && out_val, "topk_f64: null pointer");
  const int kk = (int)(top_k < n ? top_k : n);
  if (kk > kTopkSelectMax)
    return sort_topk_rows<double>(vals, n_rows, n, row_stride, kk, out_idx, out_val, workspace, workspace_bytes,
                                as_stream(stream));
  return topk_rows<double>(vals, n_rows, n, row_stride, kk, out_idx, out_val, workspace, workspace_bytes,
                           as_stream(stream));
}

static constexpr int kMinmaxParts = 256;

extern "C" size_t hrec_fuse_workspace_bytes(int64_t n, int top_k) {
  const int64_t kk = top_k < n ? top_k : n;
  const size_t t = kk > kTopkSelectMax ? sort_topk_ws_bytes(1, n) : topk_ws_bytes(1, n, (int)kk, 8);
  return (size_t)kMinmaxParts * 4 * 8 + 64 + (size_t)n * 8 + t;
}

extern "C" int hrec_fuse_topk(const double* als, const void* tt, int tt_is_f32, int64_t n, int als_wins,
                              int top_k, int64_t* out_idx, double* out_score, double* out_fused,
                              double* out_minmax, void* workspace, size_t workspace_bytes, void* stream) {
  HREC_REQUIRE(n >= 0, "fuse_topk: negative n");
  HREC_REQUIRE(top_k >= 0, "fuse_topk: top_k must be >= 0");
  if (n == 0) return HREC_OK;
  HREC_REQUIRE(als && tt, "fuse_topk: null input");
  HREC_REQUIRE(top_k == 0 || (out_idx && out_score), "fuse_topk: null output");
  const size_t need = hrec_fuse_workspace_bytes(n, top_k);
  HREC_REQUIRE(workspace && workspace_bytes >= need, "fuse_topk: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t s = as_stream(stream);
  char* w = (char*)workspace;
  double* part = (double*)w;
  double* coef = (double*)(w + kMinmaxParts * 4 * 8);
  double* fused = out_fused ? out_fused : (double*)(w + kMinmaxParts * 4 * 8 + 64);
  char* tws = w + kMinmaxParts * 4 * 8 + 64 + (size_t)n * 8;
  const size_t tws_bytes = workspace_bytes - (kMinmaxParts * 4 * 8 + 64 + (size_t)n * 8);
  const int parts = (int)((n + 255) / 256 < kMinmaxParts ? (n + 255) / 256 : kMinmaxParts);
  hipLaunchKernelGGL(minmax_partial_kernel, dim3(parts), dim3(256), 0, s, als, tt, tt_is_f32, n, part);
  int rc = check_launch("minmax_partial_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(minmax_final_kernel, dim3(1), dim3(64), 0, s, part, parts, tt_is_f32, coef,
                     out_minmax);
  rc = check_launch("minmax_final_kernel");
  if (rc) return rc;
  // src/hybrid_system.py:69 — strict '>' picks (0.8, 0.2), else (0.2, 0.8).
  const double w0 = als_wins ? 0.8 : 0.2, w1 = als_wins ? 0.2 : 0.8;
  hipLaunchKernelGGL(fuse_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, als, tt, tt_is_f32, n,
                     coef, w0, w1, fused);
  rc = check_launch("fuse_kernel");
  if (rc || top_k == 0) return rc;
  const int kk = (int)(top_k < n ? top_k : n);
  if (kk > kTopkSelectMax) return sort_topk_rows<double>(fused, 1, n, n, kk, out_idx, out_score, tws, tws_bytes, s);
  rc = topk_rows<double>(fused, 1, n, n, kk, out_idx, out_score, tws, tws_bytes, s);
  return rc;
}

extern "C" int hrec_cosine_sim(const double* feats, int64_t n_items, int dim, const int64_t* query_rows,
                               int64_t n_query, double* out, void* stream) {
  HREC_REQUIRE(n_items >= 0 && n_query >= 0 && dim >= 1, "cosine_sim: bad shape");
  if (n_items == 0 || n_query == 0) return HREC_OK;
  HREC_REQUIRE(n_query < 65536, "cosine_sim: at most 65535 queries per call");
  HREC_REQUIRE(feats && query_rows && out, "cosine_sim: null pointer");
  const dim3 grid((unsigned)((n_items + 255) / 256), (unsigned)n_query);
  hipLaunchKernelGGL(cosine_kernel, grid, dim3(256), 0, as_stream(stream), feats, n_items, dim, query_rows, out);
  return check_launch("cosine_kernel");
}

#ifndef HREC_SCORE_UB
#define HREC_SCORE_UB 16
#endif
static constexpr int kScoreUB = HREC_SCORE_UB;
#ifndef HREC_SCORE_SAMPLE
#define HREC_SCORE_SAMPLE 2048
#endif
static constexpr int kSample = HREC_SCORE_SAMPLE;  // items scored for the survivor bound
static constexpr int kSampleUB = 4;
static constexpr int kCap = 4096;

extern "C" size_t hrec_als_score_topk_workspace_bytes(int n_users, int64_t n_items, int top_k) {
  const size_t B = (size_t)n_users;
  const int64_t S = n_items < kSample ? n_items : kSample;
  size_t b = B * (size_t)S * 4 + 256;                          // sample scores
  b += topk_ws_bytes(B, S, top_k, 4) + 256;                     // sample top-k workspace
  b += B * (size_t)top_k * 12 + 256;                            // sample top-k values / indices
  b += B * (size_t)kCap * 12 + 256;                             // candidates
  b += B * 4 + 256 + 16;                                        // counters + flag
  b += topk_ws_bytes(B, kCap, top_k, 4) + 256;                  // final top-k workspace
  return b;
}

static char* carve(char*& p, size_t bytes) {
  char* r = p;
  p += (bytes + 255) & ~(size_t)255;
  return r;
}

extern "C" int hrec_als_score_topk(const float* user_factors, const int64_t* user_rows, int n_users,
                                   const float* item_factors_t, int64_t ld_items, int64_t n_items, int k, int kp,
                                   int top_k, int64_t* out_idx, float* out_val, int* overflow, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  HREC_REQUIRE(hrec_factor_ld_ok(kp), "als_score_topk: kp must be 16, 32, 64, 96, 128, 192 or 256");
  HREC_REQUIRE(k >= 1 && k <= kp, "als_score_topk: need 1 <= k <= kp");
  HREC_REQUIRE(n_users >= 0 && n_users < 65536 && n_items >= 0, "als_score_topk: bad shape");
  HREC_REQUIRE(ld_items >= n_items && ld_items % 4 == 0 && ld_items < ((int64_t)1 << 29),
               "als_score_topk: ld_items must be >= n_items, %% 4 and < 2^29");
  HREC_REQUIRE(top_k >= 1 && top_k <= 1024, "als_score_topk: top_k must be in [1, 1024]");
  if (n_users == 0 || n_items == 0) return HREC_OK;
  HREC_REQUIRE(user_factors && user_rows && item_factors_t && out_idx && out_val && overflow && workspace,
               "als_score_topk: null pointer");
  const size_t need = hrec_als_score_topk_workspace_bytes(n_users, n_items, top_k);
  HREC_REQUIRE(workspace_bytes >= need, "als_score_topk: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t s = as_stream(stream);
  const int kk = (int)(top_k < n_items ? top_k : n_items);
  char* p = (char*)workspace;
  const int64_t S = n_items < kSample ? n_items : kSample;
  float* samp = (float*)carve(p, (size_t)n_users * S * 4);
  char* tws = carve(p, topk_ws_bytes(n_users, S, kk, 4));
  float* sv = (float*)carve(p, (size_t)n_users * kk * 4);
  int64_t* si = (int64_t*)carve(p, (size_t)n_users * kk * 8);
  float* cv = (float*)carve(p, (size_t)n_users * kCap * 4);
  int64_t* ci = (int64_t*)carve(p, (size_t)n_users * kCap * 8);
  int* cn = (int*)carve(p, (size_t)n_users * 4 + 16);
  char* fws = carve(p, topk_ws_bytes(n_users, kCap, kk, 4));
  const dim3 blk(256);
  const unsigned gy = (unsigned)((n_users + kScoreUB - 1) / kScoreUB);
  if (hipMemsetAsync(overflow, 0, sizeof(int), s) != hipSuccess) return check_launch("score_topk memset");
  if (n_items <= kSample) {  // small: score everything, exact top-k
    hipLaunchKernelGGL((als_score_fast_kernel<kScoreUB, false>), dim3(gy, (unsigned)((n_items + 1023) / 1024)), blk,
                       0, s, user_factors, user_rows, n_users, item_factors_t, ld_items, n_items, k, kp, samp,
                       nullptr, 0, 0, nullptr, nullptr, nullptr, nullptr);
    int rc = check_launch("als_score_fast_kernel");
    if (rc) return rc;
    return topk_rows<float>(samp, n_users, n_items, n_items, kk, out_idx, out_val, tws, (size_t)1 << 62, s);
  }
  // 1) thresholds: the kk-th best of the first S items bounds the final kk-th from below
  //    (4 users per block: the sample is too small to fill the chip with 16)
  hipLaunchKernelGGL((als_score_fast_kernel<kSampleUB, false>),
                     dim3((unsigned)((n_users + kSampleUB - 1) / kSampleUB), (unsigned)((S + 1023) / 1024)), blk, 0,
                     s, user_factors, user_rows, n_users, item_factors_t, ld_items, S, k, kp, samp, nullptr, 0, 0,
                     nullptr, nullptr, nullptr, nullptr);
  int rc = check_launch("als_score_fast_kernel(sample)");
  if (rc) return rc;
  const float* thr = sv + (kk - 1);
  int thr_stride = kk;
  if (kk <= 64) {  // a lower bound suffices: the 64 lane maxima's kk-th
    // (also zeroes the survivor counters: no separate memset launch)
    hipLaunchKernelGGL(sample_threshold_kernel, dim3((unsigned)((n_users + 3) / 4)), dim3(256), 0, s, samp,
                       (int64_t)n_users, S, kk, sv, cn);
    rc = check_launch("sample_threshold_kernel");
    thr = sv;
    thr_stride = 1;
  } else {
    rc = topk_rows<float>(samp, n_users, S, S, kk, si, sv, tws, (size_t)1 << 62, s);
    if (rc == HREC_OK && hipMemsetAsync(cn, 0, (size_t)n_users * 4, s) != hipSuccess)
      return check_launch("score_topk memset");
  }
  if (rc) return rc;
  // 2) fused score + filter over all items; a user whose survivors exceed
  //    kCap raises *overflow from inside the filter (the caller falls back)
  hipLaunchKernelGGL((als_score_fast_kernel<kScoreUB, true>), dim3(gy, (unsigned)((n_items + 1023) / 1024)), blk, 0,
                     s, user_factors, user_rows, n_users, item_factors_t, ld_items, n_items, k, kp, nullptr,
                     thr, thr_stride, kCap, cv, ci, cn, overflow);
  rc = check_launch("als_score_fast_kernel(filter)");
  if (rc) return rc;
  // 3) exact stable top-k over the candidates (original item index breaks ties)
  return topk_rows<float>(cv, n_users, kCap, kCap, kk, out_idx, out_val, fws, (size_t)1 << 62, s, ci, cn);
}

// ---------------------------------------------------- K2p: pruned ALS top-k
// hrec_als_score_topk's result (the stable top-k of the JVM-exact scores)
// without the exact chain over every pair: the scores are first bounded on
// the bf16 matrix cores, and the exact chain runs only for the pairs the
// bound cannot rule out.
//   bf16 operands (8 significant bits, round to nearest even: |x - bf16(x)|
//   <= 2^-8 |x|; e.g. 1 + 2^-8 + 2^-20 -> 1 + 2^-7) give products within
//   (2^-7 + 2^-16) |u_c v_c| of the exact ones, so s~ = sum uh_c vh_c has
//   |s~ - u.v| <= (2^-7 + 2^-16 + k 2^-24 (1 + 2^-6)) sum |u_c v_c| (the f32
//   accumulation of k exact bf16 products, any order), and the JVM chain is
//   within 2k 2^-24 sum |u_c v_c| of u.v; for k <= 256 both fit in
//   E_b = (2^-7 + 2^-13) ||u_b|| max_j ||v_j|| (2^-16 + 3 * 256 * 2^-24 <
//   2^-13; + 1e-30 for products the matrix cores may flush).
//   1. tau_b: the kk-th best s~ over the first 8192 items (bf16 dot on the
//      matrix cores, the fused path's lane-maxima bound) minus E_b, rounded
//      down: kk items have chain >= s~ - E_b >= tau_b, so the kk-th best
//      chain over all items is >= tau_b;
//   2. the bf16 filter (als_bound_filter_kernel) at tau_b - E_b keeps
//      every item whose chain can reach tau_b;
//   3. the JVM chain over the kept items; those >= tau_b are the candidates,
//      a superset of the top kk, ranked by the same stable top-k as the
//      fused path (ties -> smaller item).
// Users whose bound is not finite (a non-finite factor anywhere) or whose
// kept list overflows raise *overflow: the caller's fallback (the
// materialised scores + hrec_topk_f32) answers the call, as for the fused
// path's list overflow. Unknown users (row < 0) keep no candidates, as there.
constexpr double kPruneRel = 0x1p-7 + 0x1p-13;
constexpr double kPruneAbs = 1e-30;
// items of the bf16 sample bound: kk <= 64 takes the first 32768 items'
// wave-tile maxima (no score matrix; 8192 / 16384 / 32768 items -> 105 /
// 96 / 94 us per 1024 x 100k call: a larger sample leaves fewer pairs to the
// filter), kk > 64 the exact kk-th of the first 8192 items' scores (a
// materialised [B][8192] sample: 4096 / 8192 / 16384 / 32768 items measured
// 160 / 144 / 145 / 153 us before the maxima form)
constexpr int kPruneSampleMax = 32768;
constexpr int kPruneSample = 8192;
// resident users per block of the sample's dot (the full 128 KiB of users
// leaves 16 blocks for 8192 items: 64 -> 144 us, 128 -> 148, 256 -> 154;
// the filter over all items keeps the kernel's own tile, capping it measured
// no faster)
constexpr int kPruneSampleUB = 64;

__device__ __forceinline__ float pr_up(double x) {
  float f = (float)x;
  if ((double)f < x) f = nextafterf(f, INFINITY);
  return f;
}
__device__ __forceinline__ float pr_down(double x) {
  float f = (float)x;
  if ((double)f > x) f = nextafterf(f, -INFINITY);
  return f;
}
__device__ __forceinline__ uint16_t pr_bf16(float v) {  // round to nearest even (NaN stays NaN)
  const uint32_t x = __float_as_uint(v);
  if ((x & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((x >> 16) | 0x40u);
  return (uint16_t)((x + 0x7fffu + ((x >> 16) & 1u)) >> 16);
}

// Item operand: bf16 rows [N][dk] (zero beyond k) and the largest row norm
// rounded up (+inf for a non-finite value), one thread per row.
__global__ __launch_bounds__(256) void als_items_bf16_kernel(const float* __restrict__ V, int64_t ldv, int64_t N,
                                                             int k, int dk, uint16_t* __restrict__ out,
                                                             unsigned* __restrict__ max_norm) {
  const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
  double ss = 0.0;
  bool bad = false;
  if (row < N) {
    uint32_t* o = reinterpret_cast<uint32_t*>(out + row * dk);
    for (int c = 0; c < dk; c += 2) {
      const float v0 = c < k ? V[row * ldv + c] : 0.f;
      const float v1 = c + 1 < k ? V[row * ldv + c + 1] : 0.f;
      ss += (double)v0 * v0 + (double)v1 * v1;
      bad = bad || !isfinite(v0) || !isfinite(v1);
      o[c >> 1] = (uint32_t)pr_bf16(v0) | ((uint32_t)pr_bf16(v1) << 16);
    }
  }
  const double nrm = sqrt(ss) * (1.0 + 1e-6);
  unsigned f = __float_as_uint((bad || !(nrm < 0x1p60)) ? INFINITY : pr_up(nrm));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned o = (unsigned)__shfl_xor((int)f, off, kWave);
    f = o > f ? o : f;  // non-negative floats order as their bits
  }
  if ((threadIdx.x & 63) == 0) atomicMax(max_norm, f);
}

// Per user (one wave): the bf16 user operand and E_b (+inf: no usable bound,
// NaN: unknown user).
__global__ __launch_bounds__(256) void als_prune_user_kernel(const float* __restrict__ U, int kp,
                                                             const int64_t* __restrict__ user_rows, int n_users,
                                                             int k, int dk, const float* __restrict__ max_norm,
                                                             uint16_t* __restrict__ uop, double* __restrict__ err,
                                                             int* __restrict__ overflow) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x == 0) *overflow = 0;  // the call's first kernel (no memset launch)
  if (b >= n_users) return;  // wave-uniform
  const int64_t r = user_rows[b];
  double ss = 0.0;
  bool bad = false;
  for (int c = lane; c < dk; c += 64) {
    const float v = (r >= 0 && c < k) ? U[r * kp + c] : 0.f;
    ss += (double)v * v;
    bad = bad || !isfinite(v);
    uop[(int64_t)b * dk + c] = pr_bf16(v);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    ss += __shfl_xor(ss, off, kWave);
    bad = bad || __shfl_xor((int)bad, off, kWave);
  }
  if (lane == 0) {
    const double e = kPruneRel * (sqrt(ss) * (1.0 + 1e-6)) * (double)max_norm[0] + kPruneAbs;
    err[b] = r < 0 ? __builtin_nan("") : ((bad || !(e < 0x1p100)) ? INFINITY : e);
  }
}

// Per user: tau_b = down(t_b - E_b) for the exact test, down(tau_b - E_b)
// for the bf16 filter; the candidate counter zeroed.
__device__ __forceinline__ void pr_bounds(int b, double t, const double* __restrict__ err, float* __restrict__ tau,
                                          float* __restrict__ thr2, int* __restrict__ cn,
                                          int* __restrict__ overflow) {
  cn[b] = 0;
  const double e = err[b];
  float t1 = INFINITY, t2 = INFINITY;  // unknown user / no bound: nothing passes
  if (e == e) {
    const double lo1 = t - e;
    const double lo2 = (double)pr_down(lo1) - e;
    if (isfinite(t) && isfinite(e) && isfinite(lo2)) {
      t1 = pr_down(lo1);
      t2 = pr_down(lo2);
      if (!isfinite(t2)) t2 = -FLT_MAX;  // below every finite f32 score
      if (!isfinite(t1)) t1 = -FLT_MAX;
    } else {
      atomicOr(overflow, 1);  // no usable bound: the caller's exact fallback
    }
  }
  tau[b] = t1;
  thr2[b] = t2;
}

__global__ __launch_bounds__(256) void als_prune_thr_kernel(int n_users, const float* __restrict__ thr,
                                                            int thr_stride, const double* __restrict__ err,
                                                            float* __restrict__ tau, float* __restrict__ thr2,
                                                            int* __restrict__ cn, int* __restrict__ overflow) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= n_users) return;
  pr_bounds(b, thr[(int64_t)b * thr_stride], err, tau, thr2, cn, overflow);
}

// kk <= 64: sample_threshold_kernel's lane-maxima bound over the wave-tile
// maxima and the bounds above in one launch (one wave per user; zeroes the
// filter's counter too).
__global__ __launch_bounds__(256) void als_prune_sample_thr_kernel(const float* __restrict__ vals, int n_users,
                                                                   int64_t n, int kk, const double* __restrict__ err,
                                                                   float* __restrict__ tau, float* __restrict__ thr2,
                                                                   int* __restrict__ cn, int* __restrict__ pn,
                                                                   int* __restrict__ overflow) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= n_users) return;  // wave-uniform
  const float* __restrict__ rv = vals + (int64_t)b * n;
  float m = -INFINITY;
  for (int64_t p = lane; p < n; p += 64) m = fmaxf(m, rv[p]);
  float t = -INFINITY;
  for (int r = 0; r < kk; ++r) {
    float w = m;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) w = fmaxf(w, __shfl_xor(w, off, kWave));
    t = w;
    const uint64_t hold = __ballot(m == w);  // retire one lane holding the maximum (the lowest such lane)
    if (hold && lane == __builtin_ctzll(hold)) m = -INFINITY;
  }
  if (lane == 0) {
    pn[b] = 0;
    pr_bounds(b, t, err, tau, thr2, cn, overflow);
  }
}

// The exact JVM chain for every pair the bf16 filter kept (one block per
// user; a thread per candidate; the item's row-major factors as 16-B loads),
// appended to the candidate lists when it reaches tau_b. Steps c in
// [k, 4 ceil(k / 4)) add the fused kernel's zero products (its rank loop
// runs in steps of 4). A kept list past the cap raises *overflow here.
__global__ __launch_bounds__(256) void als_rescore_kernel(const float* __restrict__ U, int kp,
                                                          const int64_t* __restrict__ user_rows, int n_users, int k,
                                                          const float* __restrict__ V, int64_t ldv,
                                                          const int64_t* __restrict__ pre_i,
                                                          const int* __restrict__ pre_n, int cap,
                                                          const float* __restrict__ tau, int kk,
                                                          float* __restrict__ cand_v, int64_t* __restrict__ cand_i,
                                                          int* __restrict__ cand_n, int* __restrict__ overflow) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float su[kScoreKMax];
  const int b = blockIdx.x;
  const int64_t r = user_rows[b];
  if (r < 0) return;  // block-uniform: no candidates were kept
  if (threadIdx.x == 0 && pre_n[b] > cap) atomicOr(overflow, 1);
  for (int c = threadIdx.x; c < kp; c += blockDim.x) su[c] = c < k ? U[r * kp + c] : 0.f;
  __syncthreads();
  const int n = pre_n[b] < cap ? pre_n[b] : cap;
  const float t = tau[b];
  const int kr = (k + 3) & ~3;
  const int lane = threadIdx.x & 63;
  const bool vec = (ldv & 3) == 0 && ((uintptr_t)V & 15) == 0;
  for (int e0 = 0; e0 < n; e0 += blockDim.x) {  // block-uniform trip count: the ballots see whole waves
    const int e = e0 + threadIdx.x;
    float acc = 0.f;
    int64_t j = -1;
    if (e < n) {
      j = pre_i[(int64_t)b * cap + e];
      const float* v = V + j * ldv;
      int c = 0;
      if (vec) {
        for (; c + 4 <= k; c += 4) {
          const float4 x = *reinterpret_cast<const float4*>(v + c);
          acc = acc + su[c] * x.x;
          acc = acc + su[c + 1] * x.y;
          acc = acc + su[c + 2] * x.z;
          acc = acc + su[c + 3] * x.w;
        }
      }
      for (; c < k; ++c) acc = acc + su[c] * v[c];
      for (; c < kr; ++c) acc = acc + 0.f * 0.f;
    }
    const bool pass = e < n && acc >= t;
    const uint64_t m = __ballot(pass);
    if (m == 0) continue;
    int base = 0;
    const int leader = __builtin_ctzll(m);
    if (lane == leader) {
      base = atomicAdd(&cand_n[b], __popcll(m));
      if (base + __popcll(m) > cap) atomicOr(overflow, 1);
    }
    base = __shfl(base, leader, kWave);
    if (pass) {
      const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (pos < cap) {
        cand_v[(int64_t)b * cap + pos] = acc;
        cand_i[(int64_t)b * cap + pos] = j;
      }
    }
  }
  // fewer than kk candidates: tau_b was above the kk-th best chain (a bound
  // slip) -> the caller's exact fallback instead of (0, -1) padding
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(&cand_n[b], 0) < kk) atomicOr(overflow, 1);
}

// 2. The bf16 bound filter: block = (UBK users staged in LDS, 64 NI items),
// wave = 16 NI items held in registers for the whole block, swept over the
// users in chunks of 64 (v_mfma_f32_16x16x32_bf16: A = items, B = users, so
// lane (g, c) holds user c and items 4 g + r). A pair passes when its s~
// reaches the user's bound; survivors are rare (~0.1 %): they are staged in
// LDS (LDS atomics) and leave at the block's end with one list reservation
// per user (a returning global atomic per survivor in the loop serialised the
// waves on its round trip: 84 us against 24 us of GEMM); a lane's passing
// pairs take one LDS reservation (a mask, then the entries), their per-user
// ranks are counted at the flush (LDS atomics per survivor in the loop: 56 us
// per launch against 46; the same launch without the survivor test: 16). Measured per
// 1024 x 100k call (whole call): 2 blocks per CU and 2048 staged survivors
// 130 us; 3 per CU / 1024 staged 138; 4 per CU 132; 1 per CU 161; the next
// tile's fragments prefetched (186 VGPRs) 175.
typedef __bf16 pr_bf8 __attribute__((ext_vector_type(8)));
__host__ __device__ constexpr int prune_filter_users(int dk) { return dk <= 64 ? 256 : (dk == 128 ? 128 : 64); }
typedef float pr_f4 __attribute__((ext_vector_type(4)));

// MAXONLY (the sample bound, step 1): no test; per (user, wave tile of 16 NI
// items) the largest s~ goes to wmax[b * n_wt + tile] — disjoint item sets,
// so the kk-th largest of those maxima is reached by kk distinct items.
template <int DK, bool MAXONLY>
__global__ __launch_bounds__(256) void als_bound_filter_kernel(const uint16_t* __restrict__ uop, int n_users,
                                                               const uint16_t* __restrict__ items, int64_t N,
                                                               const float* __restrict__ thr2, int cap,
                                                               int64_t* __restrict__ pre_i, int* __restrict__ pre_n,
                                                               float* __restrict__ wmax) {
  constexpr int KS = DK / 32;
  constexpr int NI = DK <= 64 ? 4 : (DK == 128 ? 2 : 1);
  constexpr int UBK = prune_filter_users(DK);  // <= 36 KiB of users per block
  constexpr int RB = DK * 2 + 16;  // padded LDS rows: the 16 lanes of a row group hit different banks
  constexpr int CPR = DK / 8;      // 16-B chunks per user row
  constexpr int kPer = UBK * CPR / 256;
  static_assert(kPer * 256 == UBK * CPR, "whole chunks per thread");
  constexpr int kSB = 2048;  // survivors a block stages (then one list reservation per user)
  __shared__ __attribute__((aligned(16))) char us[UBK * RB];
  __shared__ float sth[UBK];
  __shared__ int s_cnt[UBK];
  __shared__ int s_n;
  __shared__ uint32_t s_item[kSB];
  __shared__ int s_rank[kSB];
  __shared__ uint16_t s_user[kSB];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int n_ut = (n_users + UBK - 1) / UBK;
  const int ut = (int)(blockIdx.x % (unsigned)n_ut);
  const int64_t it0 = blockIdx.x / (unsigned)n_ut, it_step = gridDim.x / (unsigned)n_ut;
  const int64_t n_it = (N + 64 * NI - 1) / (64 * NI);
  const int b0 = ut * UBK;
  const int ub = n_users - b0 < UBK ? n_users - b0 : UBK;
  int4 fa[KS][NI];  // this item tile's fragments
  auto load_items = [&](int64_t it, int4 (&fi)[KS][NI]) {
    const int64_t j0 = it * (64 * NI) + 16 * NI * w;
#pragma unroll
    for (int t = 0; t < NI; ++t) {
      const int64_t j = j0 + 16 * t + c;
      const int64_t jr = j < N ? j : N - 1;  // rows past the end: a valid row, masked at the test
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        fi[ks][t] = *reinterpret_cast<const int4*>(items + jr * DK + 32 * ks + 8 * g);
    }
  };
  if (it0 < n_it) load_items(it0, fa);  // in flight while the users are staged
  {  // users -> LDS: every load of a thread in flight before its stores
    int4 v[kPer];
#pragma unroll
    for (int e = 0; e < kPer; ++e) {
      const int o = threadIdx.x + 256 * e, r = o / CPR, q = o % CPR;
      v[e] = r < ub ? *reinterpret_cast<const int4*>(uop + (int64_t)(b0 + r) * DK + 8 * q) : int4{0, 0, 0, 0};
    }
#pragma unroll
    for (int e = 0; e < kPer; ++e) {
      const int o = threadIdx.x + 256 * e, r = o / CPR, q = o % CPR;
      *reinterpret_cast<int4*>(us + r * RB + 16 * q) = v[e];
    }
  }
  for (int o = threadIdx.x; o < UBK; o += 256) {
    sth[o] = (!MAXONLY && o < ub) ? thr2[b0 + o] : __builtin_nanf("");  // MAXONLY: no bounds (thr2 null)
    s_cnt[o] = 0;
  }
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const int nch = (ub + 63) / 64;
  auto tile = [&](int64_t it, int4 (&fi)[KS][NI]) {
    if (it != it0) load_items(it, fi);
    const int64_t j0 = it * (64 * NI) + 16 * NI * w;
    for (int ch = 0; ch < nch; ++ch) {
      pr_f4 acc[4][NI];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int t = 0; t < NI; ++t) acc[u][t] = pr_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        int4 uf[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          uf[u] = *reinterpret_cast<const int4*>(us + (64 * ch + 16 * u + c) * RB + 64 * ks + 16 * g);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int t = 0; t < NI; ++t)
            acc[u][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(pr_bf8, fi[ks][t]),
                                                                __builtin_bit_cast(pr_bf8, uf[u]), acc[u][t], 0, 0,
                                                                0);
      }
      const bool full = j0 + 16 * NI <= N;  // wave-uniform: every item of the wave in range
      if constexpr (MAXONLY) {
        const int64_t n_wt = (N + 16 * NI - 1) / (16 * NI);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float mx = -INFINITY;
#pragma unroll
          for (int t = 0; t < NI; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (full || j0 + 16 * t + 4 * g + r < N) mx = fmaxf(mx, acc[u][t][r]);
          mx = fmaxf(mx, __shfl_xor(mx, 16, kWave));
          mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
          const int ul = 64 * ch + 16 * u + c;
          if (g == 0 && ul < ub && j0 < N) wmax[(int64_t)(b0 + ul) * n_wt + j0 / (16 * NI)] = mx;
        }
        continue;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int ul = 64 * ch + 16 * u + c;
        const float th = sth[ul];  // NaN (absent user): nothing passes
        float mx = -INFINITY;
        if (full) {
#pragma unroll
          for (int t = 0; t < NI; ++t)
            mx = fmaxf(mx, fmaxf(fmaxf(acc[u][t][0], acc[u][t][1]), fmaxf(acc[u][t][2], acc[u][t][3])));
        } else {
#pragma unroll
          for (int t = 0; t < NI; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (j0 + 16 * t + 4 * g + r < N) mx = fmaxf(mx, acc[u][t][r]);
        }
        if (__ballot(mx >= th) == 0) continue;
        {
          // the lane's passing (t, r) as a mask; one LDS reservation per lane
          uint32_t m = 0;
#pragma unroll
          for (int t = 0; t < NI; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (j0 + 16 * t + 4 * g + r < N && acc[u][t][r] >= th) m |= 1u << (4 * t + r);
          if (m) {
            int e = atomicAdd(&s_n, __popc(m));  // LDS
            while (m) {
              const int q = __builtin_ctz(m);
              m &= m - 1;
              const int64_t j = j0 + 16 * (q >> 2) + 4 * g + (q & 3);
              if (e < kSB) {
                s_item[e] = (uint32_t)j;
                s_user[e] = (uint16_t)ul;
              } else {  // staging full: straight to the user's list
                const int64_t b = b0 + ul;
                const int p = atomicAdd(&pre_n[b], 1);
                if (p < cap) pre_i[b * cap + p] = j;
              }
              ++e;
            }
          }
        }
      }
    }
  };
  for (int64_t it = it0; it < n_it; it += it_step) tile(it, fa);
  if constexpr (MAXONLY) return;
  // flush: one list reservation per user with staged survivors, then the entries
  __syncthreads();
  {  // ranks per user (LDS atomics, off the MFMA loop)
    const int ne0 = s_n < kSB ? s_n : kSB;
    for (int e = threadIdx.x; e < ne0; e += 256) s_rank[e] = atomicAdd(&s_cnt[s_user[e]], 1);
    __syncthreads();
  }
  for (int o = threadIdx.x; o < ub; o += 256) {
    const int k = s_cnt[o];
    s_cnt[o] = k ? atomicAdd(&pre_n[b0 + o], k) : 0;
  }
  __syncthreads();
  const int ne = s_n < kSB ? s_n : kSB;
  for (int e = threadIdx.x; e < ne; e += 256) {
    const int ul = s_user[e];
    const int p = s_cnt[ul] + s_rank[e];
    if (p < cap) pre_i[(int64_t)(b0 + ul) * cap + p] = (int64_t)s_item[e];
  }
}

// 3+4 fused for kk <= 8: the candidates stay in LDS and wave 0 ranks them
// exactly as topk_wave_kernel does (per-lane sorted lists of KK, then kk
// rounds of wave arg-best; absent entries -> (0, -1)), so the call skips the
// list round trip and the top-k launch. cand_n[b] still counts the
// candidates (the bench's diagnostics; > cap raises *overflow).
template <int KK>
__global__ __launch_bounds__(256) void als_rescore_topk_kernel(const float* __restrict__ U, int kp,
                                                               const int64_t* __restrict__ user_rows, int n_users,
                                                               int k, const float* __restrict__ V, int64_t ldv,
                                                               const int64_t* __restrict__ pre_i,
                                                               const int* __restrict__ pre_n, int cap,
                                                               const float* __restrict__ tau, int kk,
                                                               int64_t* __restrict__ out_idx,
                                                               float* __restrict__ out_val, int* __restrict__ cand_n,
                                                               int* __restrict__ overflow) {
#pragma clang fp contract(off)
  constexpr int kL = 2048;  // candidates kept in LDS (more: *overflow, the caller's fallback)
  __shared__ __attribute__((aligned(16))) float su[kScoreKMax];
  __shared__ float s_v[kL];
  __shared__ int s_j[kL];
  __shared__ int s_n;
  const int b = blockIdx.x;
  const int64_t r = user_rows[b];
  const int lane = threadIdx.x & 63;
  if (threadIdx.x == 0) s_n = 0;
  if (r >= 0) {
    if (threadIdx.x == 0 && pre_n[b] > cap) atomicOr(overflow, 1);
    for (int c = threadIdx.x; c < kp; c += blockDim.x) su[c] = c < k ? U[r * kp + c] : 0.f;
  }
  __syncthreads();
  if (r >= 0) {
    const int n = pre_n[b] < cap ? pre_n[b] : cap;
    const float t = tau[b];
    const int kr = (k + 3) & ~3;
    const bool vec = (ldv & 3) == 0 && ((uintptr_t)V & 15) == 0;
    for (int e = threadIdx.x; e < n; e += blockDim.x) {
      const int64_t j = pre_i[(int64_t)b * cap + e];
      const float* v = V + j * ldv;
      float acc = 0.f;
      int c = 0;
      if (vec) {
        for (; c + 4 <= k; c += 4) {
          const float4 x = *reinterpret_cast<const float4*>(v + c);
          acc = acc + su[c] * x.x;
          acc = acc + su[c + 1] * x.y;
          acc = acc + su[c + 2] * x.z;
          acc = acc + su[c + 3] * x.w;
        }
      }
      for (; c < k; ++c) acc = acc + su[c] * v[c];
      for (; c < kr; ++c) acc = acc + 0.f * 0.f;
      if (acc >= t) {
        const int p = atomicAdd(&s_n, 1);  // LDS
        if (p < kL) {
          s_v[p] = acc;
          s_j[p] = (int)j;
        }
      }
    }
  }
  __syncthreads();
  const int m = s_n;
  if (threadIdx.x == 0) {
    cand_n[b] = m;
    // fewer than kk candidates for a known user: tau_b was above the kk-th
    // best chain (a bound slip) -> the caller's exact fallback, never short ids
    if (m > kL || m > cap || (r >= 0 && m < kk)) atomicOr(overflow, 1);
  }
  if (threadIdx.x >= 64) return;  // wave 0 ranks
  const int mm = m < kL ? m : kL;
  float lv[KK];
  int64_t li[KK];
#pragma unroll
  for (int q = 0; q < KK; ++q) {
    lv[q] = 0.f;
    li[q] = INT64_MAX;
  }
  for (int p = lane; p < mm; p += 64) {
    float xv = s_v[p];
    int64_t xi = s_j[p];
#pragma unroll
    for (int q = 0; q < KK; ++q) {
      const bool sw = li[q] == INT64_MAX || better(xv, xi, lv[q], li[q]);
      const float tv = lv[q];
      const int64_t ti = li[q];
      lv[q] = sw ? xv : tv;
      li[q] = sw ? xi : ti;
      xv = sw ? tv : xv;
      xi = sw ? ti : xi;
      if (xi == INT64_MAX) break;
    }
  }
  for (int q = 0; q < kk; ++q) {
    const KV<float> w = wave_best(KV<float>{lv[0], li[0]});
    if (lane == 0) {
      out_val[(int64_t)b * kk + q] = w.i == INT64_MAX ? 0.f : w.v;
      out_idx[(int64_t)b * kk + q] = w.i == INT64_MAX ? -1 : w.i;
    }
    if (w.i != INT64_MAX && li[0] == w.i) {
#pragma unroll
      for (int x = 0; x + 1 < KK; ++x) {
        lv[x] = lv[x + 1];
        li[x] = li[x + 1];
      }
      li[KK - 1] = INT64_MAX;
    }
  }
}

// The exact fallback of the pruned top-k for kk <= 8, on the device: when
// *gate != 0 (a user overflowed a list or had no finite bound), every user's
// stable top-kk of the JVM chain over ALL items — the chain of
// als_rescore_topk_kernel (and of the fused path), one block per user, a
// sorted list of KK per thread, then wave and block merges by arg-best rounds
// (ties -> smaller item, NaN last). An unknown user (row < 0) gets the
// pruned path's answer for it, no candidates: (0, -1) entries. Gate 0:
// every block returns after one load (no host round trip decides the
// fallback).
template <int KK>
__global__ __launch_bounds__(256) void als_exact_topk_kernel(const float* __restrict__ U, int kp,
                                                             const int64_t* __restrict__ user_rows, int n_users,
                                                             int k, const float* __restrict__ V, int64_t ldv,
                                                             int64_t N, int kk, const int* __restrict__ gate,
                                                             int64_t* __restrict__ out_idx,
                                                             float* __restrict__ out_val) {
#pragma clang fp contract(off)
  if (*gate == 0) return;  // block-uniform
  __shared__ __attribute__((aligned(16))) float su[kScoreKMax];
  __shared__ float s_v[4 * KK];
  __shared__ int64_t s_i[4 * KK];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kr = (k + 3) & ~3;
  const bool vec = (ldv & 3) == 0 && ((uintptr_t)V & 15) == 0;
  for (int b = blockIdx.x; b < n_users; b += gridDim.x) {  // block-uniform trip count
    const int64_t r = user_rows[b];
    if (r < 0) {
      for (int q = threadIdx.x; q < kk; q += blockDim.x) {
        out_val[(int64_t)b * kk + q] = 0.f;
        out_idx[(int64_t)b * kk + q] = -1;
      }
      continue;
    }
    __syncthreads();  // the previous user's readers of su / s_v are done
    for (int c = threadIdx.x; c < kp; c += blockDim.x) su[c] = c < k ? U[r * kp + c] : 0.f;
    __syncthreads();
    float lv[KK];
    int64_t li[KK];
#pragma unroll
    for (int q = 0; q < KK; ++q) {
      lv[q] = 0.f;
      li[q] = INT64_MAX;
    }
    for (int64_t j = threadIdx.x; j < N; j += blockDim.x) {
      float acc = 0.f;
      const float* v = V + j * ldv;
      int c = 0;
      if (vec) {
        for (; c + 4 <= k; c += 4) {
          const float4 x = *reinterpret_cast<const float4*>(v + c);
          acc = acc + su[c] * x.x;
          acc = acc + su[c + 1] * x.y;
          acc = acc + su[c + 2] * x.z;
          acc = acc + su[c + 3] * x.w;
        }
      }
      for (; c < k; ++c) acc = acc + su[c] * v[c];
      for (; c < kr; ++c) acc = acc + 0.f * 0.f;
      float xv = acc;
      int64_t xi = j;
#pragma unroll
      for (int q = 0; q < KK; ++q) {
        const bool sw = li[q] == INT64_MAX || better(xv, xi, lv[q], li[q]);
        const float tv = lv[q];
        const int64_t ti = li[q];
        lv[q] = sw ? xv : tv;
        li[q] = sw ? xi : ti;
        xv = sw ? tv : xv;
        xi = sw ? ti : xi;
      }
    }
    // each wave's best kk -> LDS, then wave 0 merges the four lists
    for (int q = 0; q < kk; ++q) {
      const KV<float> x = wave_best(KV<float>{lv[0], li[0]});
      if (lane == 0) {
        s_v[w * KK + q] = x.v;
        s_i[w * KK + q] = x.i;
      }
      if (x.i != INT64_MAX && li[0] == x.i) {
#pragma unroll
        for (int e = 0; e + 1 < KK; ++e) {
          lv[e] = lv[e + 1];
          li[e] = li[e + 1];
        }
        li[KK - 1] = INT64_MAX;
      }
    }
    __syncthreads();
    if (w == 0) {
      KV<float> m{0.f, INT64_MAX};
      if (lane < 4 * KK && lane % KK < kk) m = KV<float>{s_v[lane], s_i[lane]};
      for (int q = 0; q < kk; ++q) {
        const KV<float> x = wave_best(m);
        if (lane == 0) {
          out_val[(int64_t)b * kk + q] = x.i == INT64_MAX ? 0.f : x.v;
          out_idx[(int64_t)b * kk + q] = x.i == INT64_MAX ? -1 : x.i;
        }
        if (x.i != INT64_MAX && m.i == x.i) m.i = INT64_MAX;
      }
    }
  }
}

template <bool MAXONLY>
static int bound_filter_launch(int dk, dim3 grid, hipStream_t s, const uint16_t* uop, int n_users,
                               const uint16_t* items, int64_t N, const float* thr2, int cap, int64_t* pre_i,
                               int* pre_n, float* wmax) {
  switch (dk) {
    case 32: hipLaunchKernelGGL((als_bound_filter_kernel<32, MAXONLY>), grid, dim3(256), 0, s, uop, n_users, items, N,
                                thr2, cap, pre_i, pre_n, wmax); break;
    case 64: hipLaunchKernelGGL((als_bound_filter_kernel<64, MAXONLY>), grid, dim3(256), 0, s, uop, n_users, items, N,
                                thr2, cap, pre_i, pre_n, wmax); break;
    case 128: hipLaunchKernelGGL((als_bound_filter_kernel<128, MAXONLY>), grid, dim3(256), 0, s, uop, n_users, items,
                                 N, thr2, cap, pre_i, pre_n, wmax); break;
    default: hipLaunchKernelGGL((als_bound_filter_kernel<256, MAXONLY>), grid, dim3(256), 0, s, uop, n_users, items,
                                N, thr2, cap, pre_i, pre_n, wmax); break;
  }
  return check_launch("als_bound_filter_kernel");
}

// blocks of the bound filter over n items: two per CU, each walking its user
// tile over every (grid / n_ut)-th item tile (the staged users serve several)
static dim3 bound_filter_grid(int dk, int n_users, int64_t n) {
  const int64_t n_ut = (n_users + prune_filter_users(dk) - 1) / prune_filter_users(dk);
  const int per = dk <= 64 ? 256 : (dk == 128 ? 128 : 64);  // items per block round
  const int64_t n_it = (n + per - 1) / per;
  int64_t per_ut = (512 + n_ut - 1) / n_ut;
  if (per_ut > n_it) per_ut = n_it;
  return dim3((unsigned)(n_ut * per_ut));
}

static int prune_dk(int k) { return k <= 32 ? 32 : (k <= 64 ? 64 : (k <= 128 ? 128 : 256)); }

extern "C" size_t hrec_als_items_bf16_bytes(int64_t n_items, int k) {
  const int64_t n = n_items > 0 ? n_items : 0;
  return (((size_t)n * prune_dk(k) * 2 + 255) & ~(size_t)255) + 256;
}

extern "C" int hrec_als_items_bf16(const float* item_factors, int64_t ld_v, int64_t n_items, int k, void* out,
                                   size_t out_bytes, void* stream) {
  HREC_REQUIRE(k >= 1 && k <= kScoreKMax && n_items >= 0 && ld_v >= k, "als_items_bf16: bad shape");
  HREC_REQUIRE(out && out_bytes >= hrec_als_items_bf16_bytes(n_items, k) && ((uintptr_t)out & 255) == 0,
               "als_items_bf16: output must be 256-B aligned, %zu bytes", hrec_als_items_bf16_bytes(n_items, k));
  HREC_REQUIRE(n_items == 0 || item_factors, "als_items_bf16: null factors");
  hipStream_t s = as_stream(stream);
  const int dk = prune_dk(k);
  unsigned* nrm = reinterpret_cast<unsigned*>(static_cast<char*>(out) + hrec_als_items_bf16_bytes(n_items, k) - 256);
  if (hipMemsetAsync(nrm, 0, 4, s) != hipSuccess) return check_launch("als_items_bf16: memset");
  if (n_items == 0) return HREC_OK;
  hipLaunchKernelGGL(als_items_bf16_kernel, dim3((unsigned)((n_items + 255) / 256)), dim3(256), 0, s, item_factors,
                     ld_v, n_items, k, dk, static_cast<uint16_t*>(out), nrm);
  return check_launch("als_items_bf16_kernel");
}

// Workspace of the pruned path, in carve order
// (hrec_als_score_topk_pruned_counts reads the two counters).
struct PruneWs {
  float* samp;   // [B][S] bf16 sample scores
  char* tws;     // sample top-k workspace (kk > 64)
  float* sv;     // [B][kk] the sample's bound(s)
  int64_t* si;   // [B][kk]
  double* err;   // [B] E_b
  float* tau;    // [B]
  float* thr2;   // [B]
  uint16_t* uop; // [B][dk]
  int64_t* pi;   // [B][cap] the bf16 filter's kept items
  int* pn;       // [B]
  float* cv;     // [B][cap] candidates (chain >= tau)
  int64_t* ci;
  int* cn;       // [B]
  char* fws;     // final top-k workspace
  size_t total;
};

static PruneWs prune_layout(char* base, int B, int64_t N, int kk, int dk) {
  PruneWs w{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* r = base ? base + off : nullptr;
    off += (bytes + 255) & ~(size_t)255;
    return r;
  };
  const int64_t S = N < kPruneSample ? N : kPruneSample;
  w.samp = (float*)take((size_t)B * S * 4);
  w.tws = take(topk_ws_bytes(B, S, kk, 4));
  w.sv = (float*)take((size_t)B * kk * 4);
  w.si = (int64_t*)take((size_t)B * kk * 8);
  w.err = (double*)take((size_t)B * 8);
  w.tau = (float*)take((size_t)B * 4);
  w.thr2 = (float*)take((size_t)B * 4);
  w.uop = (uint16_t*)take((size_t)B * dk * 2);
  w.pi = (int64_t*)take((size_t)B * kCap * 8);
  w.pn = (int*)take((size_t)B * 4);
  w.cv = (float*)take((size_t)B * kCap * 4);
  w.ci = (int64_t*)take((size_t)B * kCap * 8);
  w.cn = (int*)take((size_t)B * 4);
  w.fws = take(topk_ws_bytes(B, kCap, kk, 4));
  w.total = off + 256;
  return w;
}

extern "C" size_t hrec_als_score_topk_pruned_workspace_bytes(int n_users, int64_t n_items, int top_k, int k) {
  const int B = n_users > 0 ? n_users : 0;
  const int64_t N = n_items > 0 ? n_items : 0;
  int kk = (int)(top_k < N ? top_k : N);
  kk = kk < 1 ? 1 : (kk > 1024 ? 1024 : kk);
  const size_t fused = hrec_als_score_topk_workspace_bytes(n_users, n_items, top_k);  // the small-catalogue path
  const size_t own = prune_layout(nullptr, B, N, kk, prune_dk(k)).total;
  return own > fused ? own : fused;
}

extern "C" int hrec_als_score_topk_pruned_counts(const void* workspace, int n_users, int64_t n_items, int top_k,
                                                 int k, int32_t* out, void* stream) {
  HREC_REQUIRE(workspace && out && n_users >= 0 && n_items >= 0 && k >= 1 && k <= kScoreKMax && top_k >= 1,
               "als_score_topk_pruned_counts: bad argument");
  if (n_users == 0) return HREC_OK;
  hipStream_t s = as_stream(stream);
  if (n_items <= kSample) {  // the fused path ran: no bf16 filter
    if (hipMemsetAsync(out, 0, (size_t)2 * n_users * 4, s) != hipSuccess)
      return check_launch("als_score_topk_pruned_counts: memset");
    return HREC_OK;
  }
  int kk = (int)(top_k < n_items ? top_k : n_items);
  kk = kk > 1024 ? 1024 : kk;
  const PruneWs w = prune_layout((char*)workspace, n_users, n_items, kk, prune_dk(k));
  if (hipMemcpyAsync(out, w.pn, (size_t)n_users * 4, hipMemcpyDeviceToDevice, s) != hipSuccess ||
      hipMemcpyAsync(out + n_users, w.cn, (size_t)n_users * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return check_launch("als_score_topk_pruned_counts: copy");
  return HREC_OK;
}

extern "C" int hrec_als_score_topk_pruned(const float* user_factors, const int64_t* user_rows, int n_users,
                                          const float* item_factors_t, int64_t ld_items, const float* item_factors,
                                          int64_t ld_v, const void* items_bf16, int64_t n_items, int k, int kp,
                                          int top_k, int64_t* out_idx, float* out_val, int* overflow,
                                          void* workspace, size_t workspace_bytes, void* stream) {
  HREC_REQUIRE(hrec_factor_ld_ok(kp), "als_score_topk_pruned: kp must be 16, 32, 64, 96, 128, 192 or 256");
  HREC_REQUIRE(k >= 1 && k <= kp, "als_score_topk_pruned: need 1 <= k <= kp");
  HREC_REQUIRE(n_users >= 0 && n_users < 65536 && n_items >= 0, "als_score_topk_pruned: bad shape");
  HREC_REQUIRE(ld_items >= n_items && ld_items % 4 == 0 && ld_items < ((int64_t)1 << 29),
               "als_score_topk_pruned: ld_items must be >= n_items, %% 4 and < 2^29");
  HREC_REQUIRE(ld_v >= k, "als_score_topk_pruned: ld_v must be >= k");
  HREC_REQUIRE(top_k >= 1 && top_k <= 1024, "als_score_topk_pruned: top_k must be in [1, 1024]");
  if (n_users == 0 || n_items == 0) return HREC_OK;
  HREC_REQUIRE(user_factors && user_rows && item_factors_t && item_factors && items_bf16 && out_idx && out_val &&
                   overflow && workspace,
               "als_score_topk_pruned: null pointer");
  HREC_REQUIRE(((uintptr_t)items_bf16 & 255) == 0, "als_score_topk_pruned: items_bf16 must be 256-B aligned");
  const size_t need = hrec_als_score_topk_pruned_workspace_bytes(n_users, n_items, top_k, k);
  HREC_REQUIRE(workspace_bytes >= need, "als_score_topk_pruned: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t s = as_stream(stream);
  const int kk = (int)(top_k < n_items ? top_k : n_items);
  // kk <= 8: a set *overflow is resolved here, on the device (the gated
  // exact top-k over every item), so the result is always exact
  auto exact_fallback = [&]() {
    if (kk > 8) return (int)HREC_OK;
#define HREC_EXT(KK)                                                                                             \
  hipLaunchKernelGGL(als_exact_topk_kernel<KK>, dim3((unsigned)(n_users < 512 ? n_users : 512)), dim3(256), 0, s,  \
                     user_factors, kp, user_rows, n_users, k, item_factors, ld_v, n_items, kk, overflow, out_idx,     \
                     out_val)
    if (kk <= 2) HREC_EXT(2);
    else if (kk <= 4) HREC_EXT(4);
    else HREC_EXT(8);
#undef HREC_EXT
    return check_launch("als_exact_topk_kernel");
  };
  if (n_items <= kSample) {  // small: the fused path scores everything anyway
    const int rc = hrec_als_score_topk(user_factors, user_rows, n_users, item_factors_t, ld_items, n_items, k, kp,
                                       top_k, out_idx, out_val, overflow, workspace, workspace_bytes, stream);
    return rc ? rc : exact_fallback();
  }
  const int dk = prune_dk(k);
  const PruneWs w = prune_layout((char*)workspace, n_users, n_items, kk, dk);
  const int64_t S = n_items < kPruneSample ? n_items : kPruneSample;
  const float* max_norm = reinterpret_cast<const float*>(static_cast<const char*>(items_bf16) +
                                                         hrec_als_items_bf16_bytes(n_items, k) - 256);
  // 1) bf16 user operands and E_b (and *overflow = 0); the sample's bf16 scores; its bound
  hipLaunchKernelGGL(als_prune_user_kernel, dim3((unsigned)((n_users + 3) / 4)), dim3(256), 0, s, user_factors, kp,
                     user_rows, n_users, k, dk, max_norm, w.uop, w.err, overflow);
  int rc = check_launch("als_prune_user_kernel");
  if (rc) return rc;
  if (kk <= 64) {
    // per (user, 16 NI-item wave tile) maxima of the sample (no score
    // matrix), then the kk-th of their 64 lane maxima: kk distinct items of
    // the sample reach it; zeroes pn
    const int ni = dk <= 64 ? 4 : (dk == 128 ? 2 : 1);
    const int64_t SM = n_items < kPruneSampleMax ? n_items : kPruneSampleMax;
    const int64_t n_wt = (SM + 16 * ni - 1) / (16 * ni);  // <= min(n_items, 8192) = the samp row length
    rc = bound_filter_launch<true>(dk, bound_filter_grid(dk, n_users, SM), s, w.uop, n_users,
                                   static_cast<const uint16_t*>(items_bf16), SM, nullptr, 0, nullptr, nullptr, w.samp);
    if (rc) return rc;
    hipLaunchKernelGGL(als_prune_sample_thr_kernel, dim3((unsigned)((n_users + 3) / 4)), dim3(256), 0, s, w.samp,
                       n_users, n_wt, kk, w.err, w.tau, w.thr2, w.cn, w.pn, overflow);
    rc = check_launch("als_prune_sample_thr_kernel");
    if (rc) return rc;
  } else {
    rc = dot_scores_run(w.uop, n_users, items_bf16, S, dk, 1, w.samp, S, s, kPruneSampleUB);
    if (rc) return rc;
    rc = topk_rows<float>(w.samp, n_users, S, S, kk, w.si, w.sv, w.tws, (size_t)1 << 62, s);
    if (rc == HREC_OK && hipMemsetAsync(w.pn, 0, (size_t)n_users * 4, s) != hipSuccess)
      return check_launch("score_topk_pruned memset");
    if (rc) return rc;
    hipLaunchKernelGGL(als_prune_thr_kernel, dim3((unsigned)((n_users + 255) / 256)), dim3(256), 0, s, n_users,
                       w.sv + (kk - 1), kk, w.err, w.tau, w.thr2, w.cn, overflow);
    rc = check_launch("als_prune_thr_kernel");
    if (rc) return rc;
  }
  // 2) the matrix-core filter over every item at tau_b - E_b
  {
    const dim3 grid = bound_filter_grid(dk, n_users, n_items);
    rc = bound_filter_launch<false>(dk, grid, s, w.uop, n_users, static_cast<const uint16_t*>(items_bf16), n_items,
                                    w.thr2, kCap, w.pi, w.pn, nullptr);
    if (rc) return rc;
  }
  // 3) the exact chain over the kept pairs -> candidates (chain >= tau_b);
  //    kk <= 8: ranked in the same block
  if (kk <= 8) {
#define HREC_RTK(KK)                                                                                          \
  hipLaunchKernelGGL(als_rescore_topk_kernel<KK>, dim3((unsigned)n_users), dim3(256), 0, s, user_factors, kp,      \
                     user_rows, n_users, k, item_factors, ld_v, w.pi, w.pn, kCap, w.tau, kk, out_idx, out_val, w.cn, \
                     overflow)
    if (kk <= 2) HREC_RTK(2);
    else if (kk <= 4) HREC_RTK(4);
    else HREC_RTK(8);
#undef HREC_RTK
    rc = check_launch("als_rescore_topk_kernel");
    return rc ? rc : exact_fallback();
  }
  hipLaunchKernelGGL(als_rescore_kernel, dim3((unsigned)n_users), dim3(256), 0, s, user_factors, kp, user_rows,
                     n_users, k, item_factors, ld_v, w.pi, w.pn, kCap, w.tau, kk, w.cv, w.ci, w.cn, overflow);
  rc = check_launch("als_rescore_kernel");
  if (rc) return rc;
  // 4) the same exact stable top-k over the candidates
  return topk_rows<float>(w.cv, n_users, kCap, kCap, kk, out_idx, out_val, w.fws, (size_t)1 << 62, s, w.ci, w.cn);
}

extern "C" int hrec_rows_minmax_f32(const float* x, int64_t n_rows, int64_t n, int64_t ld, float* out, void* stream) {
  HREC_REQUIRE(n_rows >= 0 && n >= 0 && ld >= n, "rows_minmax: bad shape");
  if (n_rows == 0) return HREC_OK;
  HREC_REQUIRE(n_rows < (1ll << 31), "rows_minmax: too many rows");
  HREC_REQUIRE(x && out, "rows_minmax: null pointer");
  const int vec4 = (ld % 4 == 0) && ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
  hipLaunchKernelGGL(rows_minmax_kernel, dim3((unsigned)n_rows), dim3(1024), 0, as_stream(stream), x, n, ld, vec4,
                     out);
  return check_launch("rows_minmax_kernel");
}

// Threshold-filter path (kk <= kFuseK): sample segments per row
static int64_t fuse_sample_segs(int64_t n, int /*kk*/) {
  // ~kk / G expected candidates per segment (the bound is the best of G
  // segments' kk-th best) against kFuseSlots
  const int64_t segs = (n + kFuseSeg - 1) / kFuseSeg;
  return segs < 4 ? segs : 4;
}
static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

extern "C" size_t hrec_fuse_rows_workspace_bytes(int64_t n_rows, int64_t n, int top_k) {
  const int kk = (int)(top_k < n ? top_k : n);
  if (kk >= 1 && kk <= kFuseK) {
    const int64_t segs = (n + kFuseSeg - 1) / kFuseSeg, G = fuse_sample_segs(n, kk);
    const size_t seg_path = 2 * al256((size_t)n_rows * segs * kk * 8) + topk_ws_bytes(n_rows, segs * kk, kk, 8);
    return 2 * al256((size_t)n_rows * G * kk * 8) + al256(4) + 2 * seg_path + 256;
  }
  return (size_t)n_rows * n * 8 + 256 + topk_ws_bytes(n_rows, n, top_k, 8);
}

extern "C" int hrec_fuse_rows_topk(const float* als, const float* tt, int64_t n_rows, int64_t n, int64_t ld,
                                   const float* als_minmax, const float* tt_minmax, int als_wins, int top_k,
                                   int64_t idx_offset, int64_t* out_idx, double* out_val, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  HREC_REQUIRE(n_rows >= 0 && n >= 1 && ld >= n, "fuse_rows_topk: bad shape");
  HREC_REQUIRE(n_rows < 65536, "fuse_rows_topk: at most 65535 rows per call");
  HREC_REQUIRE(top_k >= 1 && top_k <= 1024, "fuse_rows_topk: top_k must be in [1, 1024]");
  if (n_rows == 0) return HREC_OK;
  HREC_REQUIRE(als && tt && als_minmax && tt_minmax && out_idx && out_val && workspace, "fuse_rows_topk: null pointer");
  const size_t need = hrec_fuse_rows_workspace_bytes(n_rows, n, top_k);
  HREC_REQUIRE(workspace_bytes >= need, "fuse_rows_topk: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t s = as_stream(stream);
  const double w0 = als_wins ? 0.8 : 0.2, w1 = als_wins ? 0.2 : 0.8;
  const int kk = (int)(top_k < n ? top_k : n);
  int rc;
  if (kk <= kFuseK) {
    // 1. sample: the exact top-kk of each row's first G segments
    // 2. filter: every item whose fused key reaches the sample bound -> row list
    // 3. exact keyed top-kk of the lists
    // 4. (gated on overflow) the exact segment path over every segment
    const int64_t segs = (n + kFuseSeg - 1) / kFuseSeg, G = fuse_sample_segs(n, kk);
    char* p = (char*)workspace;
    auto take = [&](size_t b) { char* q = p; p += al256(b); return q; };
    double* sv = (double*)take((size_t)n_rows * G * kk * 8);
    int64_t* si = (int64_t*)take((size_t)n_rows * G * kk * 8);
    int* over = (int*)take(4);
    double* cv = (double*)take((size_t)n_rows * segs * kk * 8);
    int64_t* ci = (int64_t*)take((size_t)n_rows * segs * kk * 8);
    char* tws = take(topk_ws_bytes(n_rows, segs * kk, kk, 8));
    double* gv = (double*)take((size_t)n_rows * segs * kk * 8);
    int64_t* gi = (int64_t*)take((size_t)n_rows * segs * kk * 8);
    char* gws = p;
#define HREC_FUSE_K(K, GRID, SEGS, V, I, GATE, CLEAR)                                                           \
  case K:                                                                                                       \
    hipLaunchKernelGGL(fuse_segment_topk_kernel<K>, GRID, dim3(256), 0, s, als, tt, n, ld, SEGS, als_minmax,   \
                       tt_minmax, w0, w1, V, I, GATE, CLEAR);                                                   \
    break;
#define HREC_FUSE_SWITCH(GRID, SEGS, V, I, GATE, CLEAR)                                                          \
  switch (kk) {                                                                                                 \
    HREC_FUSE_K(1, GRID, SEGS, V, I, GATE, CLEAR) HREC_FUSE_K(2, GRID, SEGS, V, I, GATE, CLEAR)                \
    HREC_FUSE_K(3, GRID, SEGS, V, I, GATE, CLEAR) HREC_FUSE_K(4, GRID, SEGS, V, I, GATE, CLEAR)                \
    HREC_FUSE_K(5, GRID, SEGS, V, I, GATE, CLEAR) HREC_FUSE_K(6, GRID, SEGS, V, I, GATE, CLEAR)                \
    HREC_FUSE_K(7, GRID, SEGS, V, I, GATE, CLEAR) default : HREC_FUSE_K(8, GRID, SEGS, V, I, GATE, CLEAR)      \
  }
    const dim3 gs((unsigned)((G + 3) / 4), (unsigned)n_rows);
    HREC_FUSE_SWITCH(gs, G, sv, si, nullptr, over)  // also clears the overflow flag
    rc = check_launch("fuse_segment_topk_kernel (sample)");
    if (rc) return rc;
    const dim3 gf((unsigned)((segs + 3) / 4), (unsigned)n_rows);
    hipLaunchKernelGGL(fuse_filter_kernel, gf, dim3(256), 0, s, als, tt, n, ld, segs, als_minmax, tt_minmax, w0, w1,
                       sv, (int)G, kk, cv, ci, over);
    rc = check_launch("fuse_filter_kernel");
    if (rc) return rc;
    rc = topk_rows<double>(cv, n_rows, segs * kk, segs * kk, kk, out_idx, out_val, tws, (size_t)1 << 62, s, ci);
    if (rc) return rc;
    // exact path, run only if some row overflowed its list (one block per
    // row: a skipped launch costs a small grid)
    HREC_FUSE_SWITCH(dim3(1, (unsigned)n_rows), segs, gv, gi, over, nullptr)
#undef HREC_FUSE_SWITCH
#undef HREC_FUSE_K
    rc = check_launch("fuse_segment_topk_kernel (gated)");
    if (rc) return rc;
    rc = topk_rows<double>(gv, n_rows, segs * kk, segs * kk, kk, out_idx, out_val, gws, (size_t)1 << 62, s, gi,
                           nullptr, over);
  } else {
    double* fused = (double*)workspace;
    char* tws = (char*)workspace + (((size_t)n_rows * n * 8 + 255) & ~(size_t)255);
    hipLaunchKernelGGL(fuse_rows_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)n_rows), dim3(256), 0, s, als,
                       tt, n, ld, als_minmax, tt_minmax, w0, w1, fused);
    rc = check_launch("fuse_rows_kernel");
    if (rc) return rc;
    rc = topk_rows<double>(fused, n_rows, n, n, kk, out_idx, out_val, tws, (size_t)1 << 62, s);
  }
  if (rc || idx_offset == 0) return rc;
  const int64_t tot = n_rows * kk;
  hipLaunchKernelGGL(add_offset_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, out_idx, tot, idx_offset);
  return check_launch("add_offset_kernel");
}

namespace hrec {
// The exact segment path of hrec_fuse_rows_topk (kk <= kFuseK), gated on a
// device flag (launches do nothing while *gate == 0): the pruned hybrid
// top-k's fallback (csrc/hybrid_prune.hip). One block per row walks every
// segment; then the keyed top-kk of the segments' candidates.
size_t fuse_rows_exact_ws_bytes(int64_t n_rows, int64_t n, int kk) {
  const int64_t segs = (n + kFuseSeg - 1) / kFuseSeg;
  return 2 * al256((size_t)n_rows * segs * kk * 8) + topk_ws_bytes(n_rows, segs * kk, kk, 8) + 256;
}

int fuse_rows_exact(const float* als, const float* tt, int64_t n_rows, int64_t n, int64_t ld, const float* als_mm,
                    const float* tt_mm, double w0, double w1, int kk, int64_t* out_idx, double* out_val, void* ws,
                    hipStream_t s, const int* gate) {
  if (kk < 1 || kk > kFuseK) {
    set_error("fuse_rows_exact: kk must be in [1, %d]", kFuseK);
    return HREC_E_INVALID;
  }
  const int64_t segs = (n + kFuseSeg - 1) / kFuseSeg;
  char* p = (char*)ws;
  double* gv = (double*)p;
  p += al256((size_t)n_rows * segs * kk * 8);
  int64_t* gi = (int64_t*)p;
  p += al256((size_t)n_rows * segs * kk * 8);
  const dim3 grid(1, (unsigned)n_rows);
  switch (kk) {
#define HREC_FX(K)                                                                                                  \
  case K:                                                                                                           \
    hipLaunchKernelGGL(fuse_segment_topk_kernel<K>, grid, dim3(256), 0, s, als, tt, n, ld, segs, als_mm, tt_mm, w0, \
                       w1, gv, gi, gate, nullptr);                                                                  \
    break;
    HREC_FX(1) HREC_FX(2) HREC_FX(3) HREC_FX(4) HREC_FX(5) HREC_FX(6) HREC_FX(7) default : HREC_FX(8)
#undef HREC_FX
  }
  const int rc = check_launch("fuse_segment_topk_kernel (exact, gated)");
  if (rc) return rc;
  return topk_rows<double>(gv, n_rows, segs * kk, segs * kk, kk, out_idx, out_val, p, (size_t)1 << 62, s, gi, nullptr,
                           gate);
}
}  // namespace hrec

extern "C" int hrec_topk_f64_keyed(const double* vals, const int64_t* keys, int64_t n_rows, int64_t n, int top_k,
                                   int64_t* out_idx, double* out_val, void* workspace, size_t workspace_bytes,
                                   void* stream) {
  HREC_REQUIRE(n_rows >= 0 && n >= 0, "topk_f64_keyed: bad shape");
  HREC_REQUIRE(top_k >= 1 && top_k <= 1024, "topk_f64_keyed: top_k must be in [1, 1024]");
  if (n_rows == 0 || n == 0) return HREC_OK;
  HREC_REQUIRE(n_rows < 65536, "topk_f64_keyed: at most 65535 rows per call");
  HREC_REQUIRE(vals && keys && out_idx && out_val, "topk_f64_keyed: null pointer");
  const int kk = (int)(top_k < n ? top_k : n);
  HREC_REQUIRE(workspace_bytes >= topk_ws_bytes(n_rows, n, kk, 8), "topk_f64_keyed: workspace too small");
  return topk_rows<double>(vals, n_rows, n, n, kk, out_idx, out_val, workspace, workspace_bytes, as_stream(stream),
                           keys);
}
