// K9f: the hybrid recommendation of BASELINE config c5 fused on the matrix
// cores — ALS scores <u_als, v_als> and two-tower scores <u_tt, v_tt> of a
// batch of users against every item, the reference's per-model MinMaxScaler
// fusion and a stable top-k (src/hybrid_system.py:57-75, :108), without
// writing either [B, N] score matrix:
//   pass 1 (MINMAX): both GEMMs, per-user min / max of each score row
//                    (ordered-int atomics once per wave at the end);
//   pass 2 (SAMPLE): fused scores of a strided item sample -> k-th best = a
//                    lower bound of each user's k-th best fused score;
//   pass 3 (FILTER): both GEMMs again, fusion in registers, survivors of the
//                    bound appended per user; exact stable top-k of those.
// Fusion arithmetic is fuse_rows_kernel's (csrc/score.hip), contraction off:
// ALS branch in f64 from the f32 score, two-tower branch in f32 (sklearn
// keeps float32), fused = w0 * an + w1 * (double)tn. Scores accumulate in
// f32 from bf16 operands in the same MFMA k order as hrec_dot_scores, so the
// result equals the unfused bf16 path (dot scores + hrec_fuse_rows_topk)
// bit for bit.
//
// Tiling: 512-thread block = 2 (users) x 4 (items) waves, each 64 users x 32
// items as 4 x 2 tiles of v_mfma_f32_16x16x32_bf16 (A = items, B = users:
// one user per lane and user tile). Both user operand blocks sit in LDS
// (XOR-swizzled 16-B chunks); item fragments stream through a 2-step ring
// across the ALS steps, the two-tower steps and the next tile.
#include <float.h>
#include <limits.h>

#include "common.h"

// Item-fragment ring depth (steps in flight; one step = 8 MFMAs = 128
// cycles): the min/max and sample passes have registers to spare.
#ifndef HREC_HY_RING
#define HREC_HY_RING(MODE) ((MODE) == 2 ? 4 : 8)
#endif

namespace hrec {

typedef float hy_f4 __attribute__((ext_vector_type(4)));
typedef __bf16 hy_bf8 __attribute__((ext_vector_type(8)));
typedef int hy_rsrc __attribute__((ext_vector_type(4)));
__device__ hy_f4 hy_sbuf_load(hy_rsrc rsrc, int vindex, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.struct.buffer.load.v4f32");

union HyFrag {
  int4 i;
  hy_f4 f;
};

constexpr int kHyThreads = 512;
constexpr int kHyNU = 4, kHyNI = 2, kHyWU = 2, kHyWI = 4;
constexpr int kHyUsers = 16 * kHyNU * kHyWU;  // 128
constexpr int kHyItems = 16 * kHyNI * kHyWI;  // 128

enum { kHyMinMax = 0, kHySample = 1, kHyFilter = 2 };

// float <-> int key with the order of the floats (no NaN)
__device__ __forceinline__ int hy_key(float f) {
  const int b = __float_as_int(f);
  return b >= 0 ? b : b ^ 0x7fffffff;
}
__device__ __forceinline__ float hy_unkey(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7fffffff); }

template <int DK>
struct HyShape {
  static constexpr int KS = DK / 32;                    // bf16 k steps of 32
  static constexpr int kChunks = DK * 2 / 16;           // 16-B chunks per row
  static constexpr bool kSwz = kChunks >= 16;
  static constexpr int kRowB = kSwz ? kChunks * 16 : kChunks * 16 + 16;
  static constexpr int kLds = 2 * kHyUsers * kRowB;     // ALS + two-tower user rows
};

template <int DK, int MODE>
__global__ __launch_bounds__(kHyThreads) void hybrid_tile_kernel(
    const char* __restrict__ Ua, const char* __restrict__ Ut, int B, const char* __restrict__ Va,
    const char* __restrict__ Vt, int64_t n_rows, int64_t n_items, int64_t item_step, int n_ut,
    const float* __restrict__ als_mm, const float* __restrict__ tt_mm, double w0, double w1,
    int* __restrict__ mm_keys, double* __restrict__ out, int64_t ldo, const double* __restrict__ thr,
    int thr_stride, int cap, double* __restrict__ cand_v, int64_t* __restrict__ cand_i, int* __restrict__ cand_n,
    int64_t idx_offset) {
#pragma clang fp contract(off)
  using S = HyShape<DK>;
  constexpr int NU = kHyNU, NI = kHyNI, KS = S::KS;
  constexpr int P = HREC_HY_RING(MODE) < 2 * KS ? HREC_HY_RING(MODE) : 2 * KS;
  static_assert((2 * KS) % P == 0, "ring depth must divide the steps of a tile");
  __shared__ __attribute__((aligned(16))) char us[S::kLds];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int wu = w % kHyWU, wi = w / kHyWU;
  const int per_xcd = gridDim.x >> 3;
  const int lin = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  const int ut = lin % n_ut;
  const int64_t ig = lin / n_ut, n_ig = gridDim.x / n_ut;
  const int64_t n_it = (n_items + kHyItems - 1) / kHyItems;
  const int b0 = ut * kHyUsers;
  const bool active = ig < n_it;  // block-uniform; idle blocks still reach the final reduction
  if (active) {
    // stage both user blocks: batches of 8 independent 16-B loads per thread
    // in flight (a plain loop would wait out one load latency per chunk)
    constexpr int NCH = 2 * kHyUsers * S::kChunks, PER = NCH / kHyThreads, BAT = PER < 8 ? PER : 8;
    static_assert(NCH % kHyThreads == 0 && PER % BAT == 0, "staging split");
#pragma unroll
    for (int q0 = 0; q0 < PER; q0 += BAT) {
      int4 v[BAT];
#pragma unroll
      for (int j = 0; j < BAT; ++j) {
        const int o = threadIdx.x + (q0 + j) * kHyThreads;
        const int m = o / (kHyUsers * S::kChunks);
        const int r = (o / S::kChunks) % kHyUsers, q = o % S::kChunks;
        v[j] = int4{0, 0, 0, 0};
        if (b0 + r < B) v[j] = *reinterpret_cast<const int4*>((m ? Ut : Ua) + (int64_t)(b0 + r) * (DK * 2) + 16 * q);
      }
#pragma unroll
      for (int j = 0; j < BAT; ++j) {
        const int o = threadIdx.x + (q0 + j) * kHyThreads;
        const int m = o / (kHyUsers * S::kChunks);
        const int r = (o / S::kChunks) % kHyUsers, q = o % S::kChunks;
        *reinterpret_cast<int4*>(us + (m * kHyUsers + r) * S::kRowB + 16 * (S::kSwz ? q ^ (r & 15) : q)) = v[j];
      }
    }
  }
  // this lane's users: ub + 16 u (u < NU)
  const int ub = b0 + 16 * NU * wu + c;
  double ascale[NU], amin_[NU], th[NU];
  float tscale[NU], tmin_[NU];
  float amn[NU], amx[NU], tmn[NU], tmx[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    amn[u] = tmn[u] = FLT_MAX;
    amx[u] = tmx[u] = -FLT_MAX;
    ascale[u] = amin_[u] = th[u] = 0.0;
    tscale[u] = tmin_[u] = 0.f;
    const int b = ub + 16 * u;
    if (MODE != kHyMinMax && b < B) {
      const double amin = (double)als_mm[b], amax = (double)als_mm[B + b];
      double arange = amax - amin;
      if (arange < 10.0 * DBL_EPSILON) arange = 1.0;
      ascale[u] = 1.0 / arange;
      amin_[u] = 0.0 - amin * ascale[u];
      const float tmin = tt_mm[b], tmax = tt_mm[B + b];
      float trange = tmax - tmin;
      if (trange < 10.0f * FLT_EPSILON) trange = 1.0f;
      tscale[u] = 1.0f / trange;
      tmin_[u] = 0.0f - tmin * tscale[u];
    }
    if (MODE == kHyFilter) {
      double t = b < B ? thr[(int64_t)b * thr_stride] : __builtin_nan("");  // NaN: never passes
      if (b < B && t != t) t = -INFINITY;                                   // NaN bound admits all
      th[u] = t;
    }
  }
  __syncthreads();
  if (active) {
    const char* ubase_a = us + (16 * NU * wu + c) * S::kRowB;
    const char* ubase_t = ubase_a + kHyUsers * S::kRowB;
    const int xq = c ^ g;
    auto user_frag = [&](int m, int u, int ks) {
      HyFrag a;
      const int off = S::kSwz ? 16 * ((4 * ks) ^ xq) : 64 * ks + 16 * g;
      a.i = *reinterpret_cast<const int4*>((m ? ubase_t : ubase_a) + 16 * u * S::kRowB + off);
      return a;
    };
    // resources per item tile, based at the tile's first row (rows_rsrc: a
    // resource spans at most 4 GiB)
    auto rsrc_of = [&](const char* V, int64_t tile) {
      return rows_rsrc(V, tile * kHyItems * item_step, DK * 2, n_rows);
    };
    hy_rsrc ra = rsrc_of(Va, ig), rt = rsrc_of(Vt, ig), ra_n = ra, rt_n = rt;
    const int voff = 16 * g;
    auto rows_of = [&](int64_t tile, int (&vi)[NI]) {
      const int64_t jb = tile * kHyItems + 16 * NI * wi;
#pragma unroll
      for (int t = 0; t < NI; ++t) {
        const int64_t j = jb + 16 * t + c;
        vi[t] = (tile < n_it && j < n_items) ? (int)((j - tile * kHyItems) * item_step) : 0x7fffffff;  // range check -> 0
      }
    };
    // step s of a tile: s < KS from the ALS matrix, s >= KS from the two-tower one
    auto item_load = [&](int s, const int (&vi)[NI], HyFrag (&f)[NI], const hy_rsrc& a_, const hy_rsrc& t_) {
#pragma unroll
      for (int t = 0; t < NI; ++t)
        f[t].f = hy_sbuf_load(s < KS ? a_ : t_, vi[t], voff + 64 * (s < KS ? s : s - KS), 0, 0);
    };
    int vcur[NI], vnext[NI];
    rows_of(ig, vcur);
    HyFrag ring[P][NI];
#pragma unroll
    for (int q = 0; q < P; ++q) item_load(q, vcur, ring[q], ra, rt);
    HyFrag ua[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) ua[u] = user_frag(0, u, 0);
    for (int64_t it = ig; it < n_it; it += n_ig) {
      const int64_t j0 = it * kHyItems + 16 * NI * wi;
      rows_of(it + n_ig, vnext);
      ra_n = rsrc_of(Va, it + n_ig);
      rt_n = rsrc_of(Vt, it + n_ig);
      hy_f4 acc[2][NU][NI];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int u = 0; u < NU; ++u)
#pragma unroll
          for (int t = 0; t < NI; ++t) acc[m][u][t] = hy_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2 * KS; ++s) {
        const int m = s < KS ? 0 : 1;
        HyFrag b[NI], a[NU];
#pragma unroll
        for (int t = 0; t < NI; ++t) b[t] = ring[s % P][t];
        if (s + P < 2 * KS) item_load(s + P, vcur, ring[s % P], ra, rt);
        else item_load(s + P - 2 * KS, vnext, ring[s % P], ra_n, rt_n);
        // user fragments one step ahead (after the last step: step 0 of the
        // next tile — the users do not change)
        const int sn = s + 1 < 2 * KS ? s + 1 : 0;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          a[u] = ua[u];
          ua[u] = user_frag(sn < KS ? 0 : 1, u, sn < KS ? sn : sn - KS);
        }
#pragma unroll
        for (int u = 0; u < NU; ++u) {
#pragma unroll
          for (int t = 0; t < NI; ++t)
            acc[m][u][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(hy_bf8, b[t].i),
                                                                  __builtin_bit_cast(hy_bf8, a[u].i), acc[m][u][t],
                                                                  0, 0, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one next-step user read
          __builtin_amdgcn_sched_group_barrier(0x008, NI, 0);  // between MFMA pairs
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int t = 0; t < NI; ++t) vcur[t] = vnext[t];
      ra = ra_n;
      rt = rt_n;
      // C/D: lane holds user ub + 16 u, items j0 + 16 t + 4 g + r
      if constexpr (MODE == kHyMinMax) {
#pragma unroll
        for (int t = 0; t < NI; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bool ok = j0 + 16 * t + 4 * g + r < n_items;
#pragma unroll
            for (int u = 0; u < NU; ++u) {
              const float a = acc[0][u][t][r], tt = acc[1][u][t][r];
              amn[u] = ok ? fminf(amn[u], a) : amn[u];
              amx[u] = ok ? fmaxf(amx[u], a) : amx[u];
              tmn[u] = ok ? fminf(tmn[u], tt) : tmn[u];
              tmx[u] = ok ? fmaxf(tmx[u], tt) : tmx[u];
            }
          }
      } else {
        double fz[NU][NI][4];
#pragma unroll
        for (int u = 0; u < NU; ++u)
#pragma unroll
          for (int t = 0; t < NI; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const double an = (double)acc[0][u][t][r] * ascale[u] + amin_[u];
              const float tn = acc[1][u][t][r] * tscale[u] + tmin_[u];
              fz[u][t][r] = w0 * an + w1 * (double)tn;
            }
        if constexpr (MODE == kHySample) {
#pragma unroll
          for (int u = 0; u < NU; ++u) {
            const int b = ub + 16 * u;
            if (b >= B) continue;
#pragma unroll
            for (int t = 0; t < NI; ++t)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int64_t j = j0 + 16 * t + 4 * g + r;
                if (j < n_items) out[(int64_t)b * ldo + j] = fz[u][t][r];
              }
          }
        } else {
          uint64_t any = 0;
#pragma unroll
          for (int u = 0; u < NU; ++u)
#pragma unroll
            for (int t = 0; t < NI; ++t)
#pragma unroll
              for (int r = 0; r < 4; ++r) any |= __ballot(fz[u][t][r] >= th[u]);
          if (any) {
#pragma unroll
            for (int u = 0; u < NU; ++u) {
              const int b = ub + 16 * u;
#pragma unroll
              for (int t = 0; t < NI; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const int64_t j = j0 + 16 * t + 4 * g + r;
                  if (j < n_items && fz[u][t][r] >= th[u]) {
                    const int pos = atomicAdd(&cand_n[b], 1);
                    if (pos < cap) {
                      cand_v[(int64_t)b * cap + pos] = fz[u][t][r];
                      cand_i[(int64_t)b * cap + pos] = j + idx_offset;
                    }
                  }
                }
            }
          }
        }
      }
    }
  }
  if constexpr (MODE == kHyMinMax) {
    // min / max over the 4 lane groups (same user), then one atomic per user
#pragma unroll
    for (int u = 0; u < NU; ++u) {
#pragma unroll
      for (int off = 16; off < 64; off <<= 1) {
        amn[u] = fminf(amn[u], __shfl_xor(amn[u], off, kWave));
        amx[u] = fmaxf(amx[u], __shfl_xor(amx[u], off, kWave));
        tmn[u] = fminf(tmn[u], __shfl_xor(tmn[u], off, kWave));
        tmx[u] = fmaxf(tmx[u], __shfl_xor(tmx[u], off, kWave));
      }
      const int b = ub + 16 * u;
      if (g == 0 && b < B && amn[u] <= amx[u]) {
        atomicMin(&mm_keys[b], hy_key(amn[u]));
        atomicMax(&mm_keys[B + b], hy_key(amx[u]));
        atomicMin(&mm_keys[2 * B + b], hy_key(tmn[u]));
        atomicMax(&mm_keys[3 * B + b], hy_key(tmx[u]));
      }
    }
  }
}

__global__ void hy_keys_init_kernel(int* __restrict__ keys, int B) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 4 * B; i += gridDim.x * blockDim.x)
    keys[i] = ((i / B) & 1) ? INT_MIN : INT_MAX;
}

// keys [amin | amax | tmin | tmax] -> als_mm [mins | maxes], tt_mm likewise
__global__ void hy_keys_decode_kernel(const int* __restrict__ keys, int B, float* __restrict__ als_mm,
                                      float* __restrict__ tt_mm) {
  for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < B; b += gridDim.x * blockDim.x) {
    const bool seen = keys[b] != INT_MAX;  // a shard without items keeps the neutral +inf / -inf
    als_mm[b] = seen ? hy_unkey(keys[b]) : INFINITY;
    als_mm[B + b] = seen ? hy_unkey(keys[B + b]) : -INFINITY;
    tt_mm[b] = seen ? hy_unkey(keys[2 * B + b]) : INFINITY;
    tt_mm[B + b] = seen ? hy_unkey(keys[3 * B + b]) : -INFINITY;
  }
}

__global__ void hy_overflow_kernel(const int* __restrict__ cand_n, int n_users, int cap, int* __restrict__ flag) {
  for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < n_users; b += gridDim.x * blockDim.x)
    if (cand_n[b] > cap) atomicOr(flag, 1);
}

// One 512-thread block per CU (its 2 x 64 KB user block allows no second
// one): each block stages its users once and sweeps as many item tiles as
// possible with them.
static unsigned hy_grid(int n_ut, int64_t n_items) {
  const int64_t n_it = (n_items + kHyItems - 1) / kHyItems;
  int64_t m = (256 + 8 * n_ut - 1) / (8 * n_ut);
  const int64_t m_max = (n_it + 7) / 8;
  if (m > m_max) m = m_max;
  if (m < 1) m = 1;
  return (unsigned)(8 * n_ut * m);
}

template <int MODE>
static int hy_launch(const void* ua, const void* ut, int B, const void* va, const void* vt, int64_t n_rows,
                     int64_t n_items, int64_t step, int dk, const float* als_mm, const float* tt_mm, double w0,
                     double w1, int* keys, double* out, int64_t ldo, const double* thr, int thr_stride, int cap,
                     double* cv, int64_t* ci, int* cn, int64_t off, hipStream_t s) {
  const int n_ut = (B + kHyUsers - 1) / kHyUsers;
  const dim3 grid(hy_grid(n_ut, n_items)), block(kHyThreads);
  const char *a = (const char*)ua, *t = (const char*)ut, *x = (const char*)va, *y = (const char*)vt;
#define HREC_HY(DK)                                                                                            \
  hipLaunchKernelGGL((hybrid_tile_kernel<DK, MODE>), grid, block, 0, s, a, t, B, x, y, n_rows, n_items, step, n_ut, \
                     als_mm, tt_mm, w0, w1, keys, out, ldo, thr, thr_stride, cap, cv, ci, cn, off)
  switch (dk) {
    case 64: HREC_HY(64); break;
    case 128: HREC_HY(128); break;
    default: HREC_HY(256); break;
  }
#undef HREC_HY
  return check_launch("hybrid_tile_kernel");
}

// Sample S (>= 4096 strided items) and survivor capacity: about kk * n / S
// items beat the sample's k-th best; the capacity holds 8x that (>= 512),
// so small catalogues get small lists (their top-k pass is one segment).
static int64_t hy_sample(int64_t n, int kk) {
  if (n <= 8192) return n;
  const int64_t cap_max = kk <= 64 ? 8192 : 128 * (int64_t)kk;
  int64_t s = (8 * (int64_t)kk * n + cap_max - 1) / cap_max;
  if (s < 4096) s = 4096;
  return s < n ? s : n;
}
static int64_t hy_cap(int64_t n, int kk) {
  const int64_t cap_max = kk <= 64 ? 8192 : 128 * (int64_t)kk;
  const int64_t S = hy_sample(n, kk);
  int64_t cap = (8 * (int64_t)kk * n / S + 255) / 256 * 256;
  if (cap < 512) cap = 512;
  return cap < cap_max ? cap : cap_max;
}
static char* hy_carve(char*& p, size_t bytes) {
  char* r = p;
  p += (bytes + 255) & ~(size_t)255;
  return r;
}

}  // namespace hrec

using namespace hrec;

static int hy_check(const void* ua, const void* ut, int B, const void* va, const void* vt, int64_t n, int dk,
                    const char* who) {
  HREC_REQUIRE(dk == 64 || dk == 128 || dk == 256, "%s: dk must be 64, 128 or 256 (got %d)", who, dk);
  HREC_REQUIRE(B >= 0 && B < 65536 && n >= 0 && n < 0x7fffffffll, "%s: bad shape", who);
  HREC_REQUIRE(B == 0 || n == 0 || (ua && ut && va && vt), "%s: null pointer", who);
  HREC_REQUIRE((((uintptr_t)ua | (uintptr_t)ut | (uintptr_t)va | (uintptr_t)vt) & 15) == 0,
               "%s: operands must be 16-B aligned", who);
  return HREC_OK;
}

extern "C" size_t hrec_hybrid_minmax_workspace_bytes(int n_users) { return (size_t)4 * (n_users > 0 ? n_users : 0) * 4 + 256; }

extern "C" int hrec_hybrid_minmax(const void* als_user, const void* tt_user, int n_users, const void* als_item,
                                  const void* tt_item, int64_t n_items, int dk, float* als_mm, float* tt_mm,
                                  void* workspace, size_t workspace_bytes, void* stream) {
  int rc = hy_check(als_user, tt_user, n_users, als_item, tt_item, n_items, dk, "hybrid_minmax");
  if (rc) return rc;
  if (n_users == 0) return HREC_OK;
  HREC_REQUIRE(als_mm && tt_mm && workspace, "hybrid_minmax: null output");
  HREC_REQUIRE(workspace_bytes >= hrec_hybrid_minmax_workspace_bytes(n_users), "hybrid_minmax: workspace too small");
  hipStream_t s = as_stream(stream);
  int* keys = (int*)workspace;
  hipLaunchKernelGGL(hy_keys_init_kernel, dim3(64), dim3(256), 0, s, keys, n_users);
  rc = check_launch("hy_keys_init_kernel");
  if (rc) return rc;
  if (n_items > 0) {
    rc = hy_launch<kHyMinMax>(als_user, tt_user, n_users, als_item, tt_item, n_items, n_items, 1, dk, nullptr,
                              nullptr, 0.0, 0.0, keys, nullptr, 0, nullptr, 0, 0, nullptr, nullptr, nullptr, 0, s);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(hy_keys_decode_kernel, dim3(64), dim3(256), 0, s, keys, n_users, als_mm, tt_mm);
  return check_launch("hy_keys_decode_kernel");
}

extern "C" size_t hrec_hybrid_topk_workspace_bytes(int n_users, int64_t n_items, int top_k) {
  const size_t B = (size_t)(n_users > 0 ? n_users : 0);
  const int kk = (int)(top_k < n_items ? top_k : n_items);
  if (kk <= 0) return 256;
  const int64_t S = hy_sample(n_items, kk), cap = hy_cap(n_items, kk);
  size_t b = B * (size_t)S * 8 + 256;
  b += topk_ws_bytes(B, S, kk, 8) + 256;
  b += B * (size_t)kk * 16 + 512;
  b += B * (size_t)cap * 16 + 512;
  b += B * 4 + 256;
  b += topk_ws_bytes(B, cap, kk, 8) + 256;
  return b;
}

extern "C" int hrec_hybrid_topk(const void* als_user, const void* tt_user, int n_users, const void* als_item,
                                const void* tt_item, int64_t n_items, int dk, const float* als_mm,
                                const float* tt_mm, int als_wins, int top_k, const double* thr_in,
                                int64_t idx_offset, int64_t* out_idx, double* out_val, int* overflow,
                                void* workspace, size_t workspace_bytes, void* stream) {
  int rc = hy_check(als_user, tt_user, n_users, als_item, tt_item, n_items, dk, "hybrid_topk");
  if (rc) return rc;
  HREC_REQUIRE(top_k >= 1 && top_k <= 1024, "hybrid_topk: top_k must be in [1, 1024]");
  if (n_users == 0 || n_items == 0) return HREC_OK;
  HREC_REQUIRE(als_mm && tt_mm && out_idx && out_val && overflow && workspace, "hybrid_topk: null pointer");
  const size_t need = hrec_hybrid_topk_workspace_bytes(n_users, n_items, top_k);
  HREC_REQUIRE(workspace_bytes >= need, "hybrid_topk: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t s = as_stream(stream);
  // src/hybrid_system.py:69 — strict '>' picks (0.8, 0.2), else (0.2, 0.8)
  const double w0 = als_wins ? 0.8 : 0.2, w1 = als_wins ? 0.2 : 0.8;
  const int kk = (int)(top_k < n_items ? top_k : n_items);
  const int64_t S = hy_sample(n_items, kk), cap = hy_cap(n_items, kk);
  char* p = (char*)workspace;
  double* samp = (double*)hy_carve(p, (size_t)n_users * S * 8);
  char* tws = hy_carve(p, topk_ws_bytes(n_users, S, kk, 8));
  double* sv = (double*)hy_carve(p, (size_t)n_users * kk * 8);
  int64_t* si = (int64_t*)hy_carve(p, (size_t)n_users * kk * 8);
  double* cv = (double*)hy_carve(p, (size_t)n_users * cap * 8);
  int64_t* ci = (int64_t*)hy_carve(p, (size_t)n_users * cap * 8);
  int* cn = (int*)hy_carve(p, (size_t)n_users * 4);
  char* fws = hy_carve(p, topk_ws_bytes(n_users, cap, kk, 8));
  if (hipMemsetAsync(overflow, 0, sizeof(int), s) != hipSuccess) return check_launch("hybrid_topk: memset");
  if (S == n_items && thr_in == nullptr) {  // small: every fused score, exact top-k
    rc = hy_launch<kHySample>(als_user, tt_user, n_users, als_item, tt_item, n_items, n_items, 1, dk, als_mm, tt_mm,
                              w0, w1, nullptr, samp, n_items, nullptr, 0, 0, nullptr, nullptr, nullptr, 0, s);
    if (rc) return rc;
    rc = topk_rows<double>(samp, n_users, n_items, n_items, kk, out_idx, out_val, tws, (size_t)1 << 62, s);
  } else {
    const double* thr = thr_in;
    int thr_stride = 1;
    if (thr == nullptr) {
      rc = hy_launch<kHySample>(als_user, tt_user, n_users, als_item, tt_item, n_items, S, n_items / S, dk, als_mm,
                                tt_mm, w0, w1, nullptr, samp, S, nullptr, 0, 0, nullptr, nullptr, nullptr, 0, s);
      if (rc) return rc;
      rc = topk_rows<double>(samp, n_users, S, S, kk, si, sv, tws, (size_t)1 << 62, s);
      if (rc) return rc;
      thr = sv + (kk - 1);
      thr_stride = kk;
    }
    if (hipMemsetAsync(cn, 0, (size_t)n_users * 4, s) != hipSuccess)
      return check_launch("hybrid_topk: memset");
    rc = hy_launch<kHyFilter>(als_user, tt_user, n_users, als_item, tt_item, n_items, n_items, 1, dk, als_mm, tt_mm,
                              w0, w1, nullptr, nullptr, 0, thr, thr_stride, (int)cap, cv, ci, cn, 0, s);
    if (rc) return rc;
    hipLaunchKernelGGL(hy_overflow_kernel, dim3(64), dim3(256), 0, s, cn, n_users, (int)cap, overflow);
    rc = check_launch("hy_overflow_kernel");
    if (rc) return rc;
    rc = topk_rows<double>(cv, n_users, cap, cap, kk, out_idx, out_val, fws, (size_t)1 << 62, s, ci, cn);
  }
  if (rc || idx_offset == 0) return rc;
  // shift the (non-empty) ids of this item shard
  return offset_ids(out_idx, (int64_t)n_users * kk, idx_offset, s);
}
