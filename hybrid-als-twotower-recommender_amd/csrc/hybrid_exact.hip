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
//   phase 1 (hx_stats_kernel): both models' bf16 GEMMs
//     (v_mfma_f32_32x32x16_bf16, f32 accumulation), no score stores: per user
//     and 32-item group the approximate max and min of both models (16 B per
//     user and group);
//   phase 2 (hx_user_kernel, one block per user):
//     a. exact extremes: |approx - exact| <= E = 2^-6 ||u|| max_j ||v_j||
//        (bf16 rounding of both operands: 2^-7 sum |u_c v_c|, plus the f32
//        accumulation of both forms; sum |u_c v_c| <= ||u|| ||v||), so the item
//        holding a model's exact max lies in a group whose approximate max is
//        within 2E of the approximate extreme (likewise the min). Those groups
//        are rescored exactly: the ALS JVM chain per item, the two-tower score
//        by hrec_dot_scores' own MFMA chain (v_mfma_f32_16x16x4_f32, k order
//        16 ks + 4 g + e) — the same bits as the materialised scores;
//     [with the items sharded, the caller all-reduces the extremes here (C2)]
//     b. top-k: per group an upper bound of every fused score in it
//        (hp_fuse of the approximate maxima + E, rounded up to f32: the
//        fusion arithmetic is non-decreasing in both scores); tau = the kk-th
//        best exact fused score of a few seed groups (each wave's two groups
//        with the largest bounds); every group whose bound reaches tau is
//        rescored exactly, and the exact stable top-k (ties -> smaller item)
//        is taken over those items. An item outside them has a fused score
//        below tau, under kk items already found.
//   Users with non-finite or huge norms rescore every group (same kernel);
//   users whose kk best include a NaN or fewer than kk items rescore every
//   group too (the order of NaN items is by item id over the whole shard).
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
constexpr double kHxRel = 0x1p-6;
constexpr double kHxAbs = 1e-30;  // denormal products the matrix cores may flush
constexpr double kHxHuge = 0x1p60;  // a bound above this (or non-finite): rescore every group
constexpr int kHxThreads1 = 256;
constexpr int kHxThreads2 = 512;

template <int DK>
struct HxShape {
  static constexpr int KS = DK / 16;               // 32x32x16 k-steps
  static constexpr int kRowB = DK * 2 + 16;        // LDS bytes per staged user row
  static constexpr int UB = DK == 64 ? 256 : 128;  // users per tile (2 x UB rows: <= 74 KB of LDS)
  static constexpr int NI = DK == 64 ? 2 : 1;      // 32-item tiles per wave slice (VGPR budget)
  static constexpr int kSlice = 32 * NI;
  static constexpr int kBlockItems = (kHxThreads1 / 64) * kSlice;
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

// 0. bf16 user operands [2][B][DK]: the ALS rows als_users[rows[b]] (a row
// outside [0, n_rows) reads as NaN, as hrec_als_score's unknown users), the
// two-tower rows; columns >= width zero.
__global__ __launch_bounds__(128) void hx_user_ops_kernel(const float* __restrict__ U, int64_t ldu,
                                                          const int64_t* __restrict__ rows, int64_t n_rows, int ka,
                                                          const float* __restrict__ T, int64_t ldt, int kt, int B,
                                                          int dk, uint16_t* __restrict__ uop) {
  const int b = blockIdx.x, m = blockIdx.y;
  int64_t r = b;
  bool bad = false;
  if (m == 0 && rows) {
    r = rows[b];
    bad = r < 0 || r >= n_rows;
  }
  const float* src = m ? T + (int64_t)b * ldt : U + (bad ? 0 : r) * ldu;
  const int w = m ? kt : ka;
  uint16_t* out = uop + ((int64_t)m * B + b) * dk;
  for (int c = threadIdx.x; c < dk; c += blockDim.x) {
    float v = 0.f;
    if (c < w) v = bad ? __builtin_nanf("") : src[c];
    out[c] = (uint16_t)hp_bf16(v);
  }
}

// Item-side operands (once per shard): bf16 rows [2][N][dk] (ALS, two-tower;
// zero beyond the width) and each model's largest row 2-norm rounded up
// (+inf when a row holds a non-finite value or the norm is huge). One wave per
// (row, model).
__global__ __launch_bounds__(256) void hx_prepare_kernel(const float* __restrict__ A, int64_t lda, int ka,
                                                         const float* __restrict__ T, int64_t ldt, int kt,
                                                         int64_t N, int dk, uint16_t* __restrict__ out,
                                                         unsigned* __restrict__ norms) {
  const int64_t wid = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wid >= 2 * N) return;  // wave-uniform
  const int m = (int)(wid & 1);
  const int64_t row = wid >> 1;
  const float* src = m ? T + row * ldt : A + row * lda;
  const int w = m ? kt : ka;
  double ss = 0.0;
  bool bad = false;
  for (int c = lane; c < dk; c += 64) {
    const float v = c < w ? src[c] : 0.f;
    out[((int64_t)m * N + row) * dk + c] = (uint16_t)hp_bf16(v);
    ss += (double)v * (double)v;
    bad = bad || !isfinite(v);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, kWave);
  const bool any_bad = __ballot(bad) != 0;
  if (lane == 0) {
    const double nrm = sqrt(ss) * (1.0 + 1e-6);
    const float f = (any_bad || !(nrm < kHxHuge)) ? INFINITY : hx_up(nrm);
    atomicMax(&norms[m], __float_as_uint(f));  // non-negative floats order as their bits
  }
}

// 1. Phase 1: block = (user tile of UB users, kBlockItems items); each wave
// owns one slice of NI 32-item tiles, keeps its item fragments (both models,
// every k-step) in registers and sweeps the tile's users in chunks of 32 from
// LDS. MFMA roles: A = items (32 rows), B = users (32 columns), so lane (h, c)
// holds user c and items 8 q + 4 h + r (register 4 q + r). Per (user, group):
// [max, min] of each model's approximate scores (fmaxf / fminf: NaN-free,
// like hrec_rows_minmax_f32), one 16-B record.
template <int DK>
__global__ __launch_bounds__(kHxThreads1) void hx_stats_kernel(const uint16_t* __restrict__ uop, int B, int n_ut,
                                                               const char* __restrict__ items, int64_t N, int G,
                                                               float* __restrict__ stats) {
  using S = HxShape<DK>;
  constexpr int KS = S::KS, NI = S::NI, UB = S::UB, kRowB = S::kRowB;
  __shared__ __attribute__((aligned(16))) char us[2 * UB * kRowB];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int ut = (int)(blockIdx.x % (unsigned)n_ut);
  const int64_t i0 = (int64_t)(blockIdx.x / (unsigned)n_ut) * S::kBlockItems;
  const int64_t jb = i0 + (int64_t)S::kSlice * w;
  const int b0 = ut * UB;
  const int ub = B - b0 < UB ? B - b0 : UB;
  const char* ia = items;                              // ALS operand [N][DK]
  const char* it = items + (size_t)N * (DK * 2);      // two-tower operand [N][DK]
  const hrec_rsrc_t ra = rows_rsrc(ia, i0, DK * 2, N), rt = rows_rsrc(it, i0, DK * 2, N);
  // the wave's item fragments first: they arrive while the users are staged
  HxFrag fa[NI][KS], ft[NI][KS];
  const bool work = jb < N;
  if (work) {
#pragma unroll
    for (int t = 0; t < NI; ++t) {
      const int64_t j = jb + 32 * t + c;
      const int vi = j < N ? (int)(j - i0) : 0x7fffffff;  // out of range: the buffer check reads zeros
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        fa[t][ks].f = hx_sbuf_load(ra, vi, 32 * ks + 16 * h, 0, 0);
        ft[t][ks].f = hx_sbuf_load(rt, vi, 32 * ks + 16 * h, 0, 0);
      }
    }
  }
  constexpr int CPR = DK / 8;  // 16-B chunks per user row
  for (int o = threadIdx.x; o < 2 * UB * CPR; o += kHxThreads1) {
    const int m = o / (UB * CPR), rem = o % (UB * CPR), r = rem / CPR, q = rem % CPR;
    int4 v = {0, 0, 0, 0};
    if (r < ub) v = *reinterpret_cast<const int4*>(uop + ((int64_t)(m * B + b0 + r) * DK + 8 * q));
    *reinterpret_cast<int4*>(us + (m * UB + r) * kRowB + 16 * q) = v;
  }
  __syncthreads();
  if (!work) return;  // wave-uniform; no barrier follows
  const bool full = jb + S::kSlice <= N;
  for (int ch = 0; 32 * ch < ub; ++ch) {
    hx_f16 acc[2][NI];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int t = 0; t < NI; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[m][t][v] = 0.f;
    const char* ura = us + (32 * ch + c) * kRowB + 16 * h;
    const char* urt = us + (UB + 32 * ch + c) * kRowB + 16 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      HxFrag ua, uu;
      ua.i = *reinterpret_cast<const int4*>(ura + 32 * ks);
      uu.i = *reinterpret_cast<const int4*>(urt + 32 * ks);
#pragma unroll
      for (int t = 0; t < NI; ++t) {
        acc[0][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(hx_bf8, fa[t][ks].i),
                                                            __builtin_bit_cast(hx_bf8, ua.i), acc[0][t], 0, 0, 0);
        acc[1][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(hx_bf8, ft[t][ks].i),
                                                            __builtin_bit_cast(hx_bf8, uu.i), acc[1][t], 0, 0, 0);
      }
    }
    float mx[2][NI], mn[2][NI];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int t = 0; t < NI; ++t) {
        float hi = -INFINITY, lo = INFINITY;
        if (full) {
#pragma unroll
          for (int v = 0; v < 16; ++v) {
            hi = fmaxf(hi, acc[m][t][v]);
            lo = fminf(lo, acc[m][t][v]);
          }
        } else {
#pragma unroll
          for (int v = 0; v < 16; ++v)
            if (jb + 32 * t + 8 * (v >> 2) + 4 * h + (v & 3) < N) {
              hi = fmaxf(hi, acc[m][t][v]);
              lo = fminf(lo, acc[m][t][v]);
            }
        }
        mx[m][t] = hi;
        mn[m][t] = lo;
      }
    const int b = b0 + 32 * ch + c;
    // the two lane halves hold the two halves of a group: one
    // v_permlane32_swap per register pair folds them for two tiles / models
    if constexpr (NI == 2) {
      float rec[4];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const auto X = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx[m][0]), __float_as_uint(mx[m][1]), false,
                                                        false);
        const auto Y = __builtin_amdgcn_permlane32_swap(__float_as_uint(mn[m][0]), __float_as_uint(mn[m][1]), false,
                                                        false);
        rec[2 * m] = fmaxf(hx_u2f(X[0]), hx_u2f(X[1]));  // lanes < 32: tile 0, lanes >= 32: tile 1
        rec[2 * m + 1] = fminf(hx_u2f(Y[0]), hx_u2f(Y[1]));
      }
      const int64_t grp = (jb >> 5) + h;
      if (b < B && grp < G)
        *reinterpret_cast<float4*>(stats + ((int64_t)b * G + grp) * 4) = make_float4(rec[0], rec[1], rec[2], rec[3]);
    } else {
      const auto X = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx[0][0]), __float_as_uint(mx[1][0]), false,
                                                      false);
      const auto Y = __builtin_amdgcn_permlane32_swap(__float_as_uint(mn[0][0]), __float_as_uint(mn[1][0]), false,
                                                      false);
      const float hi = fmaxf(hx_u2f(X[0]), hx_u2f(X[1]));  // lanes < 32: ALS, lanes >= 32: two-tower
      const float lo = fminf(hx_u2f(Y[0]), hx_u2f(Y[1]));
      const int64_t grp = jb >> 5;
      if (b < B) *reinterpret_cast<float2*>(stats + ((int64_t)b * G + grp) * 4 + 2 * h) = make_float2(hi, lo);
    }
  }
}

struct HxArgs {
  const float* U;  // ALS user factors (rows[b] of them; width ka)
  int64_t ldu;
  const int64_t* rows;
  int64_t n_rows;
  int ka;
  const float* T;  // two-tower user vectors [B] (width kt in {32, 64, 128})
  int64_t ldt;
  int kt;
  int B;
  const float* Va;  // ALS item factor rows [N] (f32, row stride lda)
  int64_t lda;
  const float* Vt;  // two-tower item vectors [N] (f32, row stride ldv)
  int64_t ldv;
  const float* inorm;  // [2] the item operands' largest norms (hx_prepare_kernel)
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
  int* counts;  // [2][B]: groups rescored for the extremes / for the top-k
  int* flag;    // set when a user rescored every group
};

// 2. Phase 2, one 512-thread block per user. MODE 0: the exact extremes
// (mm_a / mm_t out); 1: the top-k with the given (global) extremes; 2: both
// (one shard).
template <int DK, int MODE>
__global__ __launch_bounds__(kHxThreads2) void hx_user_kernel(HxArgs a) {
#pragma clang fp contract(off)
  constexpr int KK = kHxMaxK;
  static_assert(8 * KK == 64, "one merge slot per lane of wave 0");
  __shared__ __attribute__((aligned(16))) float sua[DK];
  __shared__ __attribute__((aligned(16))) float sut[DK];
  __shared__ float sred[8][4];
  __shared__ double se[2];
  __shared__ double rv[8 * KK];
  __shared__ int64_t ri[8 * KK];
  __shared__ double s_tau;
  __shared__ int s_full, s_cnt;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int b = blockIdx.x;
  const int64_t N = a.N;
  const int G = a.G;
  const float4* st_row = reinterpret_cast<const float4*>(a.stats) + (int64_t)b * G;
  // the user's f32 rows (the exact chains read them from LDS)
  const int64_t r = a.rows ? a.rows[b] : (int64_t)b;
  const bool rok = r >= 0 && r < a.n_rows;
  for (int c = tid; c < DK; c += kHxThreads2) {
    sua[c] = c < a.ka ? (rok ? a.U[r * a.ldu + c] : __builtin_nanf("")) : 0.f;
    sut[c] = c < a.kt ? a.T[(int64_t)b * a.ldt + c] : 0.f;
  }
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  if (wv == 0) {  // E of both models (f64 norms)
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
    }
  }
  __syncthreads();
  const double Ea = se[0], Et = se[1];
  const bool bad_a = !(Ea < kHxHuge), bad_t = !(Et < kHxHuge);  // NaN / inf / huge: no bound

  // exact scores of two groups' 64 items (lane l: item l of the pair; gB < 0:
  // none), wave-uniform: the ALS JVM chain per lane, the two-tower score by
  // 4 MFMA chains of 16 items in hrec_dot_scores' k order, moved to the lanes
  auto rescore = [&](int gA, int gB, float& s_als, float& s_tt, bool& ok, int64_t& j) {
    const int gl = lane < 32 ? gA : gB;
    j = (int64_t)gl * kHxGrp + (lane & 31);
    ok = gl >= 0 && j < N;
    {  // ALS: sequential rounded products and sums over c < ka (Spark's
       // dotProduct += a(i) * b(i)); the zero-padded tail adds +-0, a no-op
      const float* vr = a.Va + (ok ? j : 0) * a.lda;
      float s = 0.f;
      for (int c0 = 0; c0 < a.ka; c0 += 64) {
        float4 v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int cq = c0 + 4 * q;
          v[q] = cq < a.ka ? *reinterpret_cast<const float4*>(vr + cq) : make_float4(0.f, 0.f, 0.f, 0.f);
          if (cq + 4 > a.ka) {  // columns >= ka: zero (whatever the padding holds)
            if (cq + 1 >= a.ka) v[q].y = 0.f;
            if (cq + 2 >= a.ka) v[q].z = 0.f;
            if (cq + 3 >= a.ka) v[q].w = 0.f;
          }
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          if (c0 + 4 * q >= a.ka) break;
          const float4 u = *reinterpret_cast<const float4*>(sua + c0 + 4 * q);
          float p = u.x * v[q].x;
          s = s + p;
          p = u.y * v[q].y;
          s = s + p;
          p = u.z * v[q].z;
          s = s + p;
          p = u.w * v[q].w;
          s = s + p;
        }
      }
      s_als = s;
    }
    {  // two-tower
      const int g = lane >> 4, cc = lane & 15;
      const int KT = a.kt >> 4;
      hp_f4 acc[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = hp_f4{0.f, 0.f, 0.f, 0.f};
      const float* rowq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gq = q < 2 ? gA : gB;
        const int64_t jq = (int64_t)gq * kHxGrp + 16 * (q & 1) + cc;
        rowq[q] = a.Vt + ((gq >= 0 && jq < N) ? jq : 0) * a.ldv + 4 * g;
      }
      for (int ks0 = 0; ks0 < KT; ks0 += 4) {
        HxFrag itf[4][4], uf[4];
#pragma unroll
        for (int kq = 0; kq < 4; ++kq) {
          if (ks0 + kq < KT) {
#pragma unroll
            for (int q = 0; q < 4; ++q) itf[q][kq].f = *reinterpret_cast<const hp_f4*>(rowq[q] + 16 * (ks0 + kq));
            uf[kq].f = *reinterpret_cast<const hp_f4*>(sut + 16 * (ks0 + kq) + 4 * g);
          }
        }
#pragma unroll
        for (int kq = 0; kq < 4; ++kq) {
          if (ks0 + kq < KT) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
              for (int q = 0; q < 4; ++q)
                acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(itf[q][kq].f[e], uf[kq].f[e], acc[q], 0, 0, 0);
          }
        }
      }
      // lane (g, cc) holds items 16 q + 4 g + r of chain q; publish item
      // 16 (cc >> 2) + 4 g + (cc & 3), then lane l reads item l
      const hp_f4& aq = (cc >> 2) == 0 ? acc[0] : ((cc >> 2) == 1 ? acc[1] : ((cc >> 2) == 2 ? acc[2] : acc[3]));
      const float pub = hp_pick(aq, cc & 3);
      const int src = 16 * ((lane >> 2) & 3) + 4 * (lane >> 4) + (lane & 3);
      s_tt = __shfl(pub, src, kWave);
    }
  };
  // every group with pred(g) rescored, two per wave call; consume(s_als,
  // s_tt, ok, j) per lane. Groups are dealt in batches of 64 per wave.
  auto sweep = [&](auto pred, auto consume) {
    int n_resc = 0;
    int carry = -1;  // a lone group waiting for a partner
    for (int base = 64 * wv; base < G; base += 64 * 8) {
      const int g = base + lane;
      const bool p = g < G && pred(g);
      uint64_t m = __ballot(p);
      n_resc += __popcll(m);
      while (m) {
        int gA = carry;
        if (gA < 0) {
          gA = base + __builtin_ctzll(m);
          m &= m - 1;
        }
        if (!m) {
          carry = gA;
          break;
        }
        const int gB = base + __builtin_ctzll(m);
        m &= m - 1;
        carry = -1;
        float sa, stt;
        bool ok;
        int64_t j;
        rescore(gA, gB, sa, stt, ok, j);
        consume(sa, stt, ok, j);
      }
    }
    if (carry >= 0) {
      float sa, stt;
      bool ok;
      int64_t j;
      rescore(carry, -1, sa, stt, ok, j);
      consume(sa, stt, ok, j);
    }
    if (lane == 0) atomicAdd(&s_cnt, n_resc);
  };
  auto block_minmax = [&](float& lo_a, float& hi_a, float& lo_t, float& hi_t) {
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
    if (lane == 0) {
      sred[wv][0] = lo_a, sred[wv][1] = hi_a, sred[wv][2] = lo_t, sred[wv][3] = hi_t;
    }
    __syncthreads();
    lo_a = sred[0][0], hi_a = sred[0][1], lo_t = sred[0][2], hi_t = sred[0][3];
#pragma unroll
    for (int q = 1; q < 8; ++q) {
      lo_a = fminf(lo_a, sred[q][0]), hi_a = fmaxf(hi_a, sred[q][1]);
      lo_t = fminf(lo_t, sred[q][2]), hi_t = fmaxf(hi_t, sred[q][3]);
    }
  };

  float amin = INFINITY, amax = -INFINITY, tmin = INFINITY, tmax = -INFINITY;
  if constexpr (MODE != 1) {
    // a. approximate extremes, then the groups that can hold an exact one
    float AMN = INFINITY, AMX = -INFINITY, TMN = INFINITY, TMX = -INFINITY;
    for (int g = tid; g < G; g += kHxThreads2) {
      const float4 x = st_row[g];
      AMX = fmaxf(AMX, x.x), AMN = fminf(AMN, x.y), TMX = fmaxf(TMX, x.z), TMN = fminf(TMN, x.w);
    }
    block_minmax(AMN, AMX, TMN, TMX);
    const bool all_a = rok && bad_a, all_t = bad_t;
    const bool use_a = rok && !bad_a && AMX >= AMN, use_t = !bad_t && TMX >= TMN;
    const float a_hi = use_a ? hx_down((double)AMX - 2.0 * Ea) : INFINITY;
    const float a_lo = use_a ? hx_up((double)AMN + 2.0 * Ea) : -INFINITY;
    const float t_hi = use_t ? hx_down((double)TMX - 2.0 * Et) : INFINITY;
    const float t_lo = use_t ? hx_up((double)TMN + 2.0 * Et) : -INFINITY;
    const bool every = all_a || all_t;
    if (every && tid == 0) *a.flag = 1;
    float lo_a = INFINITY, hi_a = -INFINITY, lo_t = INFINITY, hi_t = -INFINITY;
    sweep(
        [&](int g) {
          if (every) return true;
          const float4 x = st_row[g];
          return x.x >= a_hi || x.y <= a_lo || x.z >= t_hi || x.w <= t_lo;
        },
        [&](float sa, float stt, bool ok, int64_t) {
          if (ok) {
            lo_a = fminf(lo_a, sa), hi_a = fmaxf(hi_a, sa);
            lo_t = fminf(lo_t, stt), hi_t = fmaxf(hi_t, stt);
          }
        });
    block_minmax(lo_a, hi_a, lo_t, hi_t);
    amin = lo_a, amax = hi_a, tmin = lo_t, tmax = hi_t;
    if (tid == 0) {
      a.counts[b] = s_cnt;
      s_cnt = 0;
    }
    __syncthreads();  // s_cnt reset before the top-k sweep counts into it
    if constexpr (MODE == 0) {
      if (tid == 0) {
        a.mm_a[b] = amin, a.mm_a[a.B + b] = amax;
        a.mm_t[b] = tmin, a.mm_t[a.B + b] = tmax;
      }
      return;
    } else {
      if (tid == 0) {
        a.mm_a[b] = amin, a.mm_a[a.B + b] = amax;
        a.mm_t[b] = tmin, a.mm_t[a.B + b] = tmax;
      }
    }
  } else {
    amin = a.mm_a[b], amax = a.mm_a[a.B + b], tmin = a.mm_t[b], tmax = a.mm_t[a.B + b];
  }
  // b. the top-k
  const int kk = a.kk;
  if (!(amin <= amax) || !(tmin <= tmax)) {
    // one model has no number at all: every fused score is NaN, and NaN
    // orders by item id
    if (tid < kk) {
      a.out_idx[(int64_t)b * kk + tid] = tid < N ? tid + a.idx_offset : -1;
      a.out_val[(int64_t)b * kk + tid] = tid < N ? __builtin_nan("") : 0.0;
    }
    if (tid == 0) a.counts[a.B + b] = 0;
    return;
  }
  const HpScale sc = hp_scale(amin, amax, tmin, tmax);
  const double w0 = a.w0, w1 = a.w1;
  bool every = bad_a || bad_t || !(isfinite(amin) && isfinite(amax) && isfinite(tmin) && isfinite(tmax));
  auto ub_of = [&](int g) {
    const float4 x = st_row[g];
    return hp_fuse(sc, hx_up((double)x.x + Ea), hx_up((double)x.z + Et), w0, w1);
  };
  HpList<KK> L;
  // the lanes' lists -> each wave's best kk -> wave 0's merge: s_tau = the
  // kk-th best value, s_full = 1 when a NaN or a missing entry is among the
  // kk; the outputs written when `write`
  auto merge = [&](bool write) {
    L.wave_top(kk, lane, rv + wv * KK, ri + wv * KK);
    __syncthreads();
    if (wv == 0) {
      double v0 = 0.0;
      int64_t i0 = INT64_MAX;
      if ((lane % KK) < kk) {
        v0 = rv[lane];
        i0 = ri[lane];
      }
      bool bad = false;
      double last = -INFINITY;
      for (int q = 0; q < kk; ++q) {
        double bv = v0;
        int64_t bi = i0;
        hp_wave_best(bv, bi);
        if (bi == INT64_MAX || bv != bv) bad = true;
        if (write && lane == 0) {
          a.out_idx[(int64_t)b * kk + q] = bi == INT64_MAX ? -1 : bi + a.idx_offset;
          a.out_val[(int64_t)b * kk + q] = bi == INT64_MAX ? 0.0 : bv;
        }
        if (bi != INT64_MAX && i0 == bi) i0 = INT64_MAX;  // the owner pops its entry
        last = bv;
      }
      if (lane == 0) {
        s_full = bad ? 1 : 0;
        s_tau = bad ? -INFINITY : last;
      }
    }
    __syncthreads();
  };
  auto take = [&](float sa, float stt, bool ok, int64_t j) {
    if (ok) L.insert(hp_fuse(sc, sa, stt, w0, w1), j);
  };
  double tau = -INFINITY;
  if (!every) {
    // seeds: each wave's two groups with the largest bounds
    double bu = -INFINITY;
    int64_t bg = INT64_MAX;
    for (int g = 64 * wv + lane; g < G; g += 64 * 8) {
      const double u = ub_of(g);
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
    L.reset();
    if (g1 != INT64_MAX) {
      float sa, stt;
      bool ok;
      int64_t j;
      rescore((int)g1, g2 == INT64_MAX ? -1 : (int)g2, sa, stt, ok, j);
      take(sa, stt, ok, j);
    }
    merge(false);
    tau = s_tau;  // -inf: fewer than kk numeric seeds (every group below qualifies)
  }
  L.reset();
  sweep([&](int g) { return every || ub_of(g) >= tau; }, take);
  merge(true);
  if (s_full && !every) {  // a NaN or a missing entry among the kk: the whole shard
    every = true;
    L.reset();
    sweep([&](int) { return true; }, take);
    merge(true);
  }
  if (tid == 0) {
    a.counts[a.B + b] = s_cnt;
    if (every) *a.flag = 1;
  }
}

struct HxWs {
  uint16_t* uop;  // [2][B][dk]
  float* stats;   // [B][G][4]
  int* counts;    // [2][B]
  int* flag;
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
  w.uop = (uint16_t*)take((size_t)2 * B * dk * 2);
  w.stats = (float*)take((size_t)B * G * 16);
  w.counts = (int*)take((size_t)2 * B * 4);
  w.flag = (int*)take(4);
  w.total = off + 256;
  return w;
}

static size_t hx_items_bytes(int64_t N, int dk) { return (((size_t)2 * N * dk * 2 + 255) & ~(size_t)255) + 256; }
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
  const int64_t ka4 = (x->als_width + 3) / 4 * 4;
  HREC_REQUIRE(x->als_items_ld >= ka4 && x->als_items_ld % 4 == 0, "%s: als_items_ld must be a multiple of 4 >= %lld",
               who, (long long)ka4);
  HREC_REQUIRE(x->tt_items_ld >= x->tt_width && x->tt_items_ld % 4 == 0,
               "%s: tt_items_ld must be a multiple of 4 >= tt_width", who);
  if (x->n_users == 0 || x->n_items == 0) return HREC_OK;
  HREC_REQUIRE(x->als_users && x->tt_users && x->als_items && x->tt_items && x->prepared, "%s: null pointer", who);
  HREC_REQUIRE((((uintptr_t)x->als_items | (uintptr_t)x->tt_items | (uintptr_t)x->prepared) & 15) == 0,
               "%s: item rows / prepared operands must be 16-B aligned", who);
  return HREC_OK;
}

extern "C" size_t hrec_hybrid_exact_items_bytes(int64_t n_items, int dk) {
  return hx_items_bytes(n_items > 0 ? n_items : 0, dk);
}

extern "C" int hrec_hybrid_exact_prepare(const float* als_items, int64_t als_ld, int als_width, const float* tt_items,
                                         int64_t tt_ld, int tt_width, int64_t n_items, int dk, void* out,
                                         void* stream) {
  HREC_REQUIRE(dk == 64 || dk == 128, "hybrid_exact_prepare: dk must be 64 or 128");
  HREC_REQUIRE(n_items >= 0 && n_items < 0x7fffffffll, "hybrid_exact_prepare: bad n_items");
  HREC_REQUIRE(als_width >= 1 && als_width <= dk && tt_width >= 1 && tt_width <= dk,
               "hybrid_exact_prepare: widths must be in [1, dk]");
  HREC_REQUIRE(als_ld >= als_width && tt_ld >= tt_width, "hybrid_exact_prepare: row stride below the width");
  HREC_REQUIRE(out && ((uintptr_t)out & 15) == 0, "hybrid_exact_prepare: output must be 16-B aligned");
  hipStream_t s = as_stream(stream);
  float* norms = const_cast<float*>(hx_norms(out, n_items, dk));
  if (hipMemsetAsync(norms, 0, 8, s) != hipSuccess) return check_launch("hybrid_exact_prepare: memset");
  if (n_items == 0) return HREC_OK;
  HREC_REQUIRE(als_items && tt_items, "hybrid_exact_prepare: null pointer");
  const int64_t waves = 2 * n_items;
  hipLaunchKernelGGL(hx_prepare_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, als_items, als_ld,
                     als_width, tt_items, tt_ld, tt_width, n_items, dk, static_cast<uint16_t*>(out),
                     reinterpret_cast<unsigned*>(norms));
  return check_launch("hx_prepare_kernel");
}

extern "C" size_t hrec_hybrid_exact_workspace_bytes(int n_users, int64_t n_items, int dk) {
  return hx_layout(nullptr, n_users > 0 ? n_users : 0, n_items > 0 ? n_items : 0, dk).total;
}

// Launches up to phase 2 (mode 0 / 2) or phase 2 alone (mode 1).
static int hx_run(const hrec_hybrid_batch* x, int mode, float* als_mm, float* tt_mm, int als_wins, int top_k,
                  int64_t idx_offset, int64_t* out_idx, double* out_val, void* workspace, hipStream_t s) {
  const int B = x->n_users, dk = x->dk;
  const int64_t N = x->n_items;
  const HxWs w = hx_layout((char*)workspace, B, N, dk);
  const int G = (int)((N + kHxGrp - 1) / kHxGrp);
  const char* items = static_cast<const char*>(x->prepared);
  if (mode != 1) {
    if (hipMemsetAsync(w.flag, 0, 4, s) != hipSuccess) return check_launch("hybrid_exact: memset");
    hipLaunchKernelGGL(hx_user_ops_kernel, dim3((unsigned)B, 2), dim3(128), 0, s, x->als_users, x->als_ld,
                       x->als_rows, x->n_als_rows, x->als_width, x->tt_users, x->tt_ld, x->tt_width, B, dk, w.uop);
    int rc = check_launch("hx_user_ops_kernel");
    if (rc) return rc;
#define HREC_HX_STATS(DK)                                                                                        \
  do {                                                                                                           \
    using S = HxShape<DK>;                                                                                       \
    const int n_ut = (B + S::UB - 1) / S::UB;                                                                    \
    const int64_t n_rng = (N + S::kBlockItems - 1) / S::kBlockItems;                                             \
    hipLaunchKernelGGL(hx_stats_kernel<DK>, dim3((unsigned)(n_ut * n_rng)), dim3(kHxThreads1), 0, s, w.uop, B,     \
                       n_ut, items, N, G, w.stats);                                                              \
  } while (0)
    if (dk == 64) HREC_HX_STATS(64); else HREC_HX_STATS(128);
#undef HREC_HX_STATS
    rc = check_launch("hx_stats_kernel");
    if (rc) return rc;
  }
  HxArgs a{};
  a.U = x->als_users, a.ldu = x->als_ld, a.rows = x->als_rows, a.n_rows = x->n_als_rows, a.ka = x->als_width;
  a.T = x->tt_users, a.ldt = x->tt_ld, a.kt = x->tt_width, a.B = B;
  a.Va = x->als_items, a.lda = x->als_items_ld, a.Vt = x->tt_items, a.ldv = x->tt_items_ld;
  a.inorm = hx_norms(x->prepared, N, dk);
  a.N = N, a.G = G, a.stats = w.stats;
  a.mm_a = als_mm, a.mm_t = tt_mm;
  // src/hybrid_system.py:69 — strict '>' picks (0.8, 0.2), else (0.2, 0.8)
  a.w0 = als_wins ? 0.8 : 0.2, a.w1 = als_wins ? 0.2 : 0.8;
  a.kk = (int)(top_k < N ? top_k : N);
  a.idx_offset = idx_offset, a.out_idx = out_idx, a.out_val = out_val;
  a.counts = w.counts, a.flag = w.flag;
#define HREC_HX_USER(DK, M) \
  hipLaunchKernelGGL((hx_user_kernel<DK, M>), dim3((unsigned)B), dim3(kHxThreads2), 0, s, a)
  if (dk == 64) {
    if (mode == 0) HREC_HX_USER(64, 0); else if (mode == 1) HREC_HX_USER(64, 1); else HREC_HX_USER(64, 2);
  } else {
    if (mode == 0) HREC_HX_USER(128, 0); else if (mode == 1) HREC_HX_USER(128, 1); else HREC_HX_USER(128, 2);
  }
#undef HREC_HX_USER
  return check_launch("hx_user_kernel");
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
