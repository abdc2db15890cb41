// K9s: both score matrices of the bf16 hybrid (BASELINE c5: rank-256 ALS
// factors and d = 256 tower vectors) in ONE launch, with the per-user
// min / max of each matrix reduced in the epilogue.
//
// Replaces, for precision "bf16", the chain the reference's
// get_hybrid_recommendations implies per user (src/hybrid_system.py:95-116:
// ALS transform + Keras Dot over every candidate, then a MinMaxScaler
// fit_transform per model, src/hybrid_system.py:57-75) up to the fusion:
// the gather of the batch's ALS user rows, their f32 -> bf16 conversion
// (round to nearest even, as hrec_f32_to_bf16), the two [B, d] x [d, N]
// GEMMs on the bf16 matrix cores (v_mfma_f32_16x16x32_bf16, f32
// accumulation, the k order of hrec_dot_scores: bit-identical scores) and
// the per-row min / max of hrec_rows_minmax_f32 (fminf / fmaxf: NaN-free
// minimum and maximum — exact under any grouping). The score matrices still
// go to HBM: the fusion's exact min-max scaling needs every row's extremes
// before any fused score exists (hrec_fuse_rows_topk reads them back).
//
// Work split: block (model, user tile, item group) stages its <= 256 users
// (128 KB at d = 256) in LDS once and owns a contiguous item range; each
// wave walks its own 16 NI-item slices of that range (no block barrier in
// the main loop, so waves of a short range simply finish early), keeping
// the slice's item fragments for the whole d in registers and sweeping the
// users in chunks of 64. The epilogue stores the tile (16-B stores) and
// folds each lane's min / max into per-user LDS slots (order-preserving
// uint keys, ds_max_u32); every block writes its partials, and a tiny
// second kernel reduces them per user (no global atomics, deterministic).
#include <float.h>

#include <type_traits>

#include "common.h"

namespace hrec {

typedef float hs_f4 __attribute__((ext_vector_type(4)));
typedef __bf16 hs_bf8 __attribute__((ext_vector_type(8)));
typedef int hs_rsrc __attribute__((ext_vector_type(4)));
__device__ hs_f4 hs_sbuf_load(hs_rsrc rsrc, int vindex, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.struct.buffer.load.v4f32");

union HsFrag {
  int4 i;
  hs_f4 f;
};

struct HybScoresArgs {
  const float* users[2];   // f32 user rows: ALS factors, two-tower user vectors
  int64_t ld[2];           // their row strides (elements)
  const int64_t* rows[2];  // row of batch user b (nullptr: row b)
  int64_t n_rows[2];       // rows of users[m]: a row outside [0, n_rows) reads as NaN
  int width[2];            // valid columns (<= DK; the operand is zero beyond)
  int B;
  const char* items[2];    // bf16 item operands [N, DK]
  int64_t N;
  float* out[2];           // score matrices [B, ldo]
  int64_t ldo;
  float* part;             // [2][G][2][B]: per-block min / max
  int* argpos;             // HS_PRUNE: [2][G][B] slice of each block's max ((jb / 16) * 4 + g), -1 = none
  const uint16_t* uop;     // optional: the batch's bf16 user operands [2][B][DK] (staged as is)
  // HS_FILTER: the heavy model hm's scores against per-(user, group) bounds
  const float* theta;      // [B][G]: a score >= theta survives; +inf / NaN: nothing of the group
  int hm;
  int cap;                 // survivor list length per user
  float* cv;               // [B][cap] survivor scores
  int64_t* ci;             // [B][cap] survivor item ids
  int* cn;                 // [B] survivors counted (zeroed by the caller; > cap: the list overflowed)
  int sbuf;                // HS_FILTER: survivors a block stages in LDS
  int fsplit;              // HS_FILTER: blocks per item group
  int G;                   // item groups per (model, user tile)
  int UB;                  // users per tile (multiple of 64)
  int n_ut;
};

#ifndef HREC_HS_ABLATE
#define HREC_HS_ABLATE 0  // timing-only builds: 1 = no score stores, 2 = and no min/max, 3 = staging only, 4 = MFMAs, no epilogue
#endif

#ifndef HREC_HS_NT
#define HREC_HS_NT 0  // 1 = non-temporal score stores
#endif

#ifndef HREC_HS_STAGE_BATCH
#define HREC_HS_STAGE_BATCH 16  // 16-B user-operand loads per thread in flight while staging
#endif
#ifndef HREC_HS_STAGE_ROT
#define HREC_HS_STAGE_ROT 1  // rotate each block's staging start (spreads the shared rows' L2 lines)
#endif

constexpr int kHsThreads = 512;
constexpr int kHsMaxUserBytes = 128 * 1024;
#ifdef HREC_HS_STAMPS
constexpr size_t kHsMaxLds = 160 * 1024 - 256;  // the stamp build's static per-wave slots take LDS too
#else
constexpr size_t kHsMaxLds = 160 * 1024;
#endif

// HS_FILTER: LDS bytes before the staged survivors (live users' rows, their
// bounds, per-user counts and overflow marks, the staging and live counters,
// the slot -> user map), 16-B aligned
__host__ __device__ inline size_t hs_filter_head(int UB, int row_b) {
  return ((size_t)UB * row_b + (size_t)UB * 16 + 8 + 15) & ~(size_t)15;
}

// f32 -> bf16 bits, round to nearest even (NaN stays NaN): hrec_f32_to_bf16.
__device__ __forceinline__ uint32_t hs_bf16(float v) {
  const uint32_t x = __float_as_uint(v);
  if ((x & 0x7fffffffu) > 0x7f800000u) return (x >> 16) | 0x40u;
  return (x + 0x7fffu + ((x >> 16) & 1u)) >> 16;
}

// The value of lane ^ 16 / lane ^ 32 by the gfx950 row / half swaps
// (v_permlane16_swap / v_permlane32_swap: VALU, no LDS round trip): with the
// same register as both operands, the swap leaves the partner's value in the
// first result for lanes with that bit set and in the second for the others.
template <typename T>
__device__ __forceinline__ T hs_xor16(T x) {
  static_assert(sizeof(T) == 4, "32-bit values");
  const uint32_t u = __builtin_bit_cast(uint32_t, x);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return __builtin_bit_cast(T, (uint32_t)((threadIdx.x & 16) ? r[0] : r[1]));
}
template <typename T>
__device__ __forceinline__ T hs_xor32(T x) {
  static_assert(sizeof(T) == 4, "32-bit values");
  const uint32_t u = __builtin_bit_cast(uint32_t, x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_bit_cast(T, (uint32_t)((threadIdx.x & 32) ? r[0] : r[1]));
}

// Order-preserving float <-> uint keys (larger float -> larger key); the
// LDS slots start at 0, below every key.
__device__ __forceinline__ uint32_t hs_key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float hs_unkey(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

template <int DK>
struct HsShape {
  static constexpr int KS = DK / 32;           // bf16 MFMA k-steps
  static constexpr int kChunks = DK * 2 / 16;  // 16-B chunks per user row
  static constexpr bool kSwz = kChunks >= 16;  // XOR-swizzled rows (as dot_res_kernel)
  static constexpr int kRowB = kSwz ? kChunks * 16 : kChunks * 16 + 16;
#ifndef HREC_HS_NI256
#define HREC_HS_NI256 2
#endif
  static constexpr int NI = DK == 64 ? 4 : (DK == 256 ? HREC_HS_NI256 : 2);  // item tiles per wave slice (VGPR budget)
  static constexpr int NU = NI == 4 ? 2 : 4;    // user tiles per chunk (NI 4: each user fragment feeds 4 MFMAs)
  // hp_bound_kernel's seed slots hold 4 NI items per group in 16 slots
  static_assert(NI >= 1 && NI <= 4, "item tiles per wave slice must be 1..4 (HREC_HS_NI256)");
};

// Modes: HS_FULL = score stores + per-block min / max (hrec_hybrid_scores);
// HS_PRUNE = no stores, min / max + the item slice holding each block's max
// (pass 1 of the pruned hybrid top-k, csrc/hybrid_prune.hip); HS_FILTER =
// the heavy model alone, survivors of the per-(user, group) bounds appended
// to per-user lists (pass 2's filter: one block per item group, so a user's
// bound is one LDS value per block and its survivors leave in one flush).
enum { HS_FULL = 0, HS_PRUNE = 1, HS_FILTER = 2 };

#ifdef HREC_HS_STAMPS
// Diagnostic builds only (plain stores per block, no contended atomics):
// [mode][block][0..3] = wave 0's s_memtime at entry, after the staging, after
// its main loop, at the end; [4 + w / 2] = (w even: low, odd: high 32 bits)
// the main-loop ticks of wave w.
constexpr int kHsStampBlocks = 1024;
__device__ unsigned long long g_hs_stamps[3][kHsStampBlocks][8];
#define HS_T() __builtin_amdgcn_s_memtime()
#endif

// NCH: user chunks of CU = 16 NU users in the tile (compile-time, so the
// per-lane running min / max of every chunk stays in registers and the last
// chunk's item refills are unconditional).
template <int DK, int NCH, int MODE>
__global__ __launch_bounds__(kHsThreads) void hyb_scores_kernel(HybScoresArgs a) {
  using S = HsShape<DK>;
  constexpr int KS = S::KS, NI = S::NI, NU = S::NU, CU = 16 * NU;
  constexpr int kRowB = S::kRowB;
#ifdef HREC_HS_STAMPS
  const unsigned long long t_start = HS_T();
#endif
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  char* us = dsm;
  uint32_t* mmk = reinterpret_cast<uint32_t*>(dsm + (size_t)a.UB * kRowB);  // [UB][2]: ~key(min), key(max)
  // HS_PRUNE: [UB] key(max) << 32 | ~slice (ds_max_u64: the larger max, then the earlier slice)
  unsigned long long* amk = reinterpret_cast<unsigned long long*>(dsm + (size_t)a.UB * kRowB + (size_t)a.UB * 8);
  // HS_FILTER (in place of the two above): [UB] bounds per slot, [UB]
  // survivor counts per user (then list bases), [UB] overflow marks per user,
  // the staging counter, the live-user counter, [UB] slot -> user, then the
  // staged survivors (meta = user << 24 | item offset in the group, score,
  // rank among the user's survivors of the block). Only the users whose
  // bound for this group is live are staged, packed into the first slots, so
  // the MFMA chunks cover ceil(live / CU) chunks instead of the whole tile.
  float* ths = reinterpret_cast<float*>(dsm + (size_t)a.UB * kRowB);
  int* cnt_l = reinterpret_cast<int*>(ths + a.UB);
  int* ovf_l = cnt_l + a.UB;
  int* bn = ovf_l + a.UB;
  int* n_live_l = bn + 1;
  int* smap = bn + 2;
  uint32_t* sb_meta = reinterpret_cast<uint32_t*>(dsm + hs_filter_head(a.UB, kRowB));
  float* sb_val = reinterpret_cast<float*>(sb_meta + a.sbuf);
  int* sb_rank = reinterpret_cast<int*>(sb_val + a.sbuf);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int model = MODE == HS_FILTER ? a.hm : (blockIdx.x & 1);
  const int rest = MODE == HS_FILTER ? (int)blockIdx.x : (int)(blockIdx.x >> 1);
  const int ut = rest % a.n_ut;
  const int grp = MODE == HS_FILTER ? rest / a.n_ut / a.fsplit : rest / a.n_ut;
  const int64_t per = ((a.N + a.G - 1) / a.G + 15) / 16 * 16;
  int64_t i0 = (int64_t)grp * per;
  int64_t i1 = i0 + per < a.N ? i0 + per : a.N;
  if constexpr (MODE == HS_FILTER) {  // part of the group: fsplit blocks share its bound
    const int part = rest / a.n_ut % a.fsplit;
    constexpr int64_t kSl = 16 * S::NI;
    const int64_t sub = (per + a.fsplit * kSl - 1) / (a.fsplit * kSl) * kSl;
    const int64_t g1 = i1;
    i0 = i0 + part * sub < g1 ? i0 + part * sub : g1;
    i1 = i0 + sub < g1 ? i0 + sub : g1;
  }
  const int b0 = ut * a.UB;
  const int ub = a.B - b0 < a.UB ? a.B - b0 : a.UB;

  // the wave's first item slice is requested before the user staging, so its
  // fragments arrive while the users are converted
  const int xq = c ^ g;
  // resource based at the block's first item (rows relative to i0: a
  // resource spans at most 4 GiB, rows_rsrc)
  const hs_rsrc rsrc = rows_rsrc(a.items[model], i0, DK * 2, a.N);
  const int voff = 16 * g;
  auto rows_of = [&](int64_t jb, int (&vi)[NI]) {
#pragma unroll
    for (int t = 0; t < NI; ++t) {
      const int64_t j = jb + 16 * t + c;
      vi[t] = j < i1 ? (int)(j - i0) : 0x7fffffff;  // out of range: the buffer check reads zeros
    }
  };
  constexpr int64_t kSlice = 16 * NI, kStride = 8 * kSlice;  // items per wave slice / per block round
  int64_t jb = i0 + kSlice * w;
  const bool work = HREC_HS_ABLATE < 3 && ub > 0 && jb < i1;
  int vnext[NI];
  rows_of(jb, vnext);
  HsFrag it_f[KS][NI];
  if (work) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int t = 0; t < NI; ++t) it_f[ks][t].f = hs_sbuf_load(rsrc, vnext[t], voff + 64 * ks, 0, 0);
  }

  // HS_FILTER: the tile's live users (bound finite, or NaN = admit all) get
  // the first slots; rows staged and MFMA chunks run for those alone
  int n_st = ub;  // rows staged (slots)
  if constexpr (MODE == HS_FILTER) {
    if (threadIdx.x == 0) *n_live_l = 0;
    __syncthreads();
    float t = __builtin_nanf("");
    int slot = -1;
    if ((int)threadIdx.x < ub) {
      t = a.theta[(int64_t)(b0 + threadIdx.x) * a.G + grp];
      // +inf: a dead (user, group) — nothing passes; NaN admits every score
      t = t == t ? (t == __builtin_inff() ? __builtin_nanf("") : t) : -__builtin_inff();
      if (t == t) slot = atomicAdd(n_live_l, 1);
    }
    __syncthreads();
    n_st = *n_live_l;
    if (slot >= 0) {
      ths[slot] = t;
      smap[slot] = (int)threadIdx.x;
    }
    for (int o = threadIdx.x; o < a.UB; o += kHsThreads) {
      if (o >= n_st) ths[o] = __builtin_nanf("");  // padding slots: nothing passes
      cnt_l[o] = 0;
      ovf_l[o] = 0;
    }
    if (threadIdx.x == 0) *bn = 0;
    __syncthreads();
  }
  auto src_row = [&](int r) { return MODE == HS_FILTER ? smap[r] : r; };

  // users of the tile -> LDS as bf16 (zero rows / columns beyond the batch /
  // width). Batches of chunks (8 floats each) per thread: all loads are
  // issued before the first conversion (16-B loads when the row allows).
  if (a.uop) {  // pre-converted rows (hp_user_ops_kernel): 16-B copies
    // every block of a launch reads the same rows: each block of an XCD
    // starts at another 1/16 of them (the same L2 lines are not requested
    // by all 32 CUs at once), and the whole tile is in flight at once at d >= 128
    const char* src = reinterpret_cast<const char*>(a.uop) + ((int64_t)model * a.B + b0) * (DK * 2);
    constexpr int kBatch = HREC_HS_STAGE_BATCH;
    const int n_chunks = (MODE == HS_FILTER ? n_st : a.UB) * S::kChunks;
    const int rot = HREC_HS_STAGE_ROT ? (int)((blockIdx.x >> 3) & 15) * (n_chunks >> 4) : 0;
    for (int o0 = threadIdx.x; o0 < n_chunks; o0 += kBatch * kHsThreads) {
      int4 v[kBatch];
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        int o = o0 + j * kHsThreads + rot;
        o = o >= n_chunks ? o - n_chunks : o;
        const int r = o / S::kChunks, q = o % S::kChunks;
        v[j] = int4{0, 0, 0, 0};
        if (o0 + j * kHsThreads < n_chunks && r < n_st)
          v[j] = *reinterpret_cast<const int4*>(src + (int64_t)src_row(r) * (DK * 2) + 16 * q);
      }
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        if (o0 + j * kHsThreads >= n_chunks) break;
        int o = o0 + j * kHsThreads + rot;
        o = o >= n_chunks ? o - n_chunks : o;
        const int r = o / S::kChunks, q = o % S::kChunks;
        *reinterpret_cast<int4*>(us + r * kRowB + 16 * (S::kSwz ? q ^ (r & 15) : q)) = v[j];
      }
    }
  } else {
    const float* src = a.users[model];
    const int64_t ld = a.ld[model];
    const int64_t* rws = a.rows[model];
    const int wd = a.width[model];
    const bool vec = (ld & 3) == 0 && ((uintptr_t)src & 15) == 0;
    constexpr int kBatch = 8;  // chunks in flight per thread (the first item slice is in flight too)
    const int n_chunks = a.UB * S::kChunks;
    for (int o0 = threadIdx.x; o0 < n_chunks; o0 += kBatch * kHsThreads) {
      float f[kBatch][8];
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        const int o = o0 + j * kHsThreads;
        const int r = o / S::kChunks, q = o % S::kChunks;
#pragma unroll
        for (int e = 0; e < 8; ++e) f[j][e] = 0.f;
        if (o < n_chunks && r < n_st && 8 * q < wd) {
          const int64_t row = rws ? rws[b0 + src_row(r)] : (int64_t)(b0 + src_row(r));
          const float* p = src + row * ld + 8 * q;
          if (row < 0 || row >= a.n_rows[model]) {  // unknown / stale row: NaN scores (as hrec_als_score's -1)
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (8 * q + e < wd) f[j][e] = __builtin_nanf("");
          } else if (vec && 8 * q + 8 <= wd) {
            const float4 x0 = *reinterpret_cast<const float4*>(p);
            const float4 x1 = *reinterpret_cast<const float4*>(p + 4);
            f[j][0] = x0.x, f[j][1] = x0.y, f[j][2] = x0.z, f[j][3] = x0.w;
            f[j][4] = x1.x, f[j][5] = x1.y, f[j][6] = x1.z, f[j][7] = x1.w;
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (8 * q + e < wd) f[j][e] = p[e];
          }
        }
      }
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        const int o = o0 + j * kHsThreads;
        if (o >= n_chunks) break;
        const int r = o / S::kChunks, q = o % S::kChunks;
        uint32_t h[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) h[e] = hs_bf16(f[j][e]);  // bf16(0.f) = 0
        const int4 v = {(int)(h[0] | (h[1] << 16)), (int)(h[2] | (h[3] << 16)), (int)(h[4] | (h[5] << 16)),
                        (int)(h[6] | (h[7] << 16))};
        *reinterpret_cast<int4*>(us + r * kRowB + 16 * (S::kSwz ? q ^ (r & 15) : q)) = v;
      }
    }
  }
  if constexpr (MODE != HS_FILTER) {
    for (int o = threadIdx.x; o < 2 * a.UB; o += kHsThreads) mmk[o] = 0u;
    if (MODE == HS_PRUNE)
      for (int o = threadIdx.x; o < a.UB; o += kHsThreads) amk[o] = 0ull;
  }
  __syncthreads();
#ifdef HREC_HS_STAMPS
  const unsigned long long t_staged = HS_T();
#endif

  // running min / max of this lane's scores per (chunk, user tile): the
  // lane's user is CU ch + 16 u + c in every slice; folded across lanes once
  float lo[NCH][NU], hi[NCH][NU];
  int hp[NCH][MODE == HS_PRUNE ? NU : 1];  // HS_PRUNE: slice (jb / 16) of the lane's max
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      lo[ch][u] = __builtin_inff(), hi[ch][u] = -__builtin_inff();
      if constexpr (MODE == HS_PRUNE) hp[ch][u] = -1;
    }
  // HS_FILTER: MFMA chunks over the live slots only
  const int nch = MODE == HS_FILTER ? (n_st + CU - 1) / CU : NCH;
  if (work && nch > 0) {
    HsFrag ua[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int off = S::kSwz ? 16 * xq : 16 * g;
      ua[u].i = *reinterpret_cast<const int4*>(us + (16 * u + c) * kRowB + off);
    }
    float* const out = a.out[model];
    for (; jb < i1; jb += kStride) {
      rows_of(jb + kStride, vnext);
      const bool full = jb + kSlice <= i1;  // wave-uniform: every item of the slice is in range
      auto user_frag = [&](int ch, int u, int ks) {
        HsFrag f;
        const int off = S::kSwz ? 16 * ((4 * ks) ^ xq) : 64 * ks + 16 * g;
        f.i = *reinterpret_cast<const int4*>(us + (CU * ch + 16 * u + c) * kRowB + off);
        return f;
      };
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        if (MODE == HS_FILTER && ch >= nch) break;
        const bool last = ch == nch - 1;
        const int ch_next = last ? 0 : ch + 1;
        hs_f4 acc[NU][NI];
#pragma unroll
        for (int u = 0; u < NU; ++u)
#pragma unroll
          for (int t = 0; t < NI; ++t) acc[u][t] = hs_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          HsFrag f[NU];
#pragma unroll
          for (int u = 0; u < NU; ++u) {
            f[u] = ua[u];
            ua[u] = ks + 1 < KS ? user_frag(ch, u, ks + 1) : user_frag(ch_next, u, 0);
          }
#pragma unroll
          for (int u = 0; u < NU; ++u)
#pragma unroll
            for (int t = 0; t < NI; ++t)
              acc[u][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(hs_bf8, it_f[ks][t].i),
                                                                  __builtin_bit_cast(hs_bf8, f[u].i), acc[u][t], 0,
                                                                  0, 0);
          if (last) {  // step ks of this slice is done: refill it with the next slice's
#pragma unroll
            for (int t = 0; t < NI; ++t) it_f[ks][t].f = hs_sbuf_load(rsrc, vnext[t], voff + 64 * ks, 0, 0);
          }
#pragma unroll
          for (int u = 0; u < NU; ++u) {
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
            __builtin_amdgcn_sched_group_barrier(0x008, NI, 0);  // MFMA
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        // C/D: lane holds user CU ch + 16 u + c, items jb + 16 t + 4 g + r
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int bl = CU * ch + 16 * u + c;
          if constexpr (MODE == HS_PRUNE) {
            // slice max first, then one compare: the lane's max and its slice
            float mx = -__builtin_inff();
            if (full) {
#pragma unroll
              for (int t = 0; t < NI; ++t) {
                lo[ch][u] = fminf(fminf(lo[ch][u], fminf(acc[u][t][0], acc[u][t][1])), fminf(acc[u][t][2], acc[u][t][3]));
                mx = fmaxf(fmaxf(mx, fmaxf(acc[u][t][0], acc[u][t][1])), fmaxf(acc[u][t][2], acc[u][t][3]));
              }
            } else {
#pragma unroll
              for (int t = 0; t < NI; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                  if (jb + 16 * t + 4 * g + r < i1) {
                    lo[ch][u] = fminf(lo[ch][u], acc[u][t][r]);
                    mx = fmaxf(mx, acc[u][t][r]);
                  }
            }
            const bool gt = mx > hi[ch][u];
            hi[ch][u] = gt ? mx : hi[ch][u];
            hp[ch][u] = gt ? (int)(jb >> 4) : hp[ch][u];
          } else if constexpr (MODE == HS_FILTER) {
            // the user's bound for this group (LDS); scores past the range are
            // never compared
            const float th = ths[bl];
            float mx = -__builtin_inff();
#pragma unroll
            for (int t = 0; t < NI; ++t)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (full || jb + 16 * t + 4 * g + r < i1) mx = fmaxf(mx, acc[u][t][r]);
            if (__ballot(mx >= th)) {  // rare: stage this lane's survivors
#pragma unroll
              for (int t = 0; t < NI; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const int64_t j = jb + 16 * t + 4 * g + r;
                  if ((full || j < i1) && acc[u][t][r] >= th) {
                    const int ul = smap[bl];  // slot -> the user's place in the tile
                    const int e = atomicAdd(bn, 1);
                    const int rk = atomicAdd(&cnt_l[ul], 1);
                    if (e < a.sbuf) {
                      sb_meta[e] = ((uint32_t)ul << 24) | (uint32_t)(j - i0);
                      sb_val[e] = acc[u][t][r];
                      sb_rank[e] = rk;
                    } else {
                      ovf_l[ul] = 1;  // staging full: the user's list is marked overflowing at the flush
                    }
                  }
                }
            }
          } else if constexpr (MODE == HS_FULL) {
            if (full) {
#pragma unroll
              for (int t = 0; t < NI; ++t) {
                lo[ch][u] = fminf(fminf(lo[ch][u], fminf(acc[u][t][0], acc[u][t][1])), fminf(acc[u][t][2], acc[u][t][3]));
                hi[ch][u] = fmaxf(fmaxf(hi[ch][u], fmaxf(acc[u][t][0], acc[u][t][1])), fmaxf(acc[u][t][2], acc[u][t][3]));
              }
            } else {
#pragma unroll
              for (int t = 0; t < NI; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                  if (jb + 16 * t + 4 * g + r < i1) {
                    lo[ch][u] = fminf(lo[ch][u], acc[u][t][r]);
                    hi[ch][u] = fmaxf(hi[ch][u], acc[u][t][r]);
                  }
            }
          }
          if (MODE == HS_FULL && HREC_HS_ABLATE == 0 && bl < ub) {
            float* o = out + (int64_t)(b0 + bl) * a.ldo;
#pragma unroll
            for (int t = 0; t < NI; ++t) {
              const int64_t j = jb + 16 * t + 4 * g;
              if (j + 3 < i1 && (a.ldo & 3) == 0) {
                if constexpr (HREC_HS_NT) {
                  __builtin_nontemporal_store(acc[u][t], reinterpret_cast<hs_f4*>(o + j));
                } else {
                  *reinterpret_cast<float4*>(o + j) =
                      make_float4(acc[u][t][0], acc[u][t][1], acc[u][t][2], acc[u][t][3]);
                }
              } else {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                  if (j + r < i1) o[j + r] = acc[u][t][r];
              }
            }
          }
        }
      }
    }
  }
#ifdef HREC_HS_STAMPS
  const unsigned long long t_loop = HS_T();
  __shared__ uint32_t s_wloop[8];
  if ((threadIdx.x & 63) == 0) s_wloop[w] = (uint32_t)(t_loop - t_staged);
  auto stamp_end = [&]() {
    if (threadIdx.x == 0 && blockIdx.x < kHsStampBlocks) {
      const unsigned long long t3 = HS_T();
      unsigned long long* o = g_hs_stamps[MODE][blockIdx.x];
      o[0] = t_start;
      o[1] = t_staged;
      o[2] = t_loop;
      o[3] = t3;
      for (int q = 0; q < 4; ++q) o[4 + q] = (unsigned long long)s_wloop[2 * q] | ((unsigned long long)s_wloop[2 * q + 1] << 32);
    }
  };
#define HS_STAMP_END() stamp_end()
#else
#define HS_STAMP_END()
#endif
  if constexpr (MODE == HS_FILTER) {
    // flush: one list reservation per user (global atomic), then the entries
    __syncthreads();
    for (int o = threadIdx.x; o < ub; o += kHsThreads) {
      const int k = cnt_l[o];
      int base = 0;
      if (ovf_l[o]) {
        atomicAdd(&a.cn[b0 + o], a.cap + 1);  // > cap: the exact path answers this user
      } else if (k > 0) {
        base = atomicAdd(&a.cn[b0 + o], k);
      }
      cnt_l[o] = ovf_l[o] ? -1 : base;
    }
    __syncthreads();
    const int ne = *bn < a.sbuf ? *bn : a.sbuf;
    for (int e = threadIdx.x; e < ne; e += kHsThreads) {
      const uint32_t m = sb_meta[e];
      const int ul = (int)(m >> 24);
      const int base = cnt_l[ul];
      if (base < 0) continue;
      const int p = base + sb_rank[e];
      if (p < a.cap) {
        const int64_t b = b0 + ul;
        a.cv[b * a.cap + p] = sb_val[e];
        a.ci[b * a.cap + p] = i0 + (int64_t)(m & 0xffffffu);
      }
    }
    HS_STAMP_END();
    return;
  }
  // fold the lanes' running min / max per user into the block's LDS slots
  if (HREC_HS_ABLATE < 2 && ub > 0) {
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int bl = CU * ch + 16 * u + c;
        float l = lo[ch][u], h = hi[ch][u];
        l = fminf(l, hs_xor16(l));
        l = fminf(l, hs_xor32(l));
        if constexpr (MODE == HS_PRUNE) {
          // (max, slice * 4 + g) of the 4 lane groups: larger max, then the smaller position
          int p = hp[ch][u] < 0 ? 0x7fffffff : hp[ch][u] * 4 + g;
          {
            const float oh = hs_xor16(h);
            const int op = hs_xor16(p);
            const bool take = oh > h || (oh == h && op < p);
            h = take ? oh : h;
            p = take ? op : p;
          }
          {
            const float oh = hs_xor32(h);
            const int op = hs_xor32(p);
            const bool take = oh > h || (oh == h && op < p);
            h = take ? oh : h;
            p = take ? op : p;
          }
          if (g == 0 && bl < ub && p != 0x7fffffff)
            atomicMax(&amk[bl], ((unsigned long long)hs_key(h) << 32) | (uint32_t)~p);
        } else {
          h = fmaxf(h, hs_xor16(h));
          h = fmaxf(h, hs_xor32(h));
        }
        if (g == 0 && bl < ub) {
          atomicMax(&mmk[2 * bl], ~hs_key(l));
          atomicMax(&mmk[2 * bl + 1], hs_key(h));
        }
      }
  }
  __syncthreads();
  for (int o = threadIdx.x; o < ub; o += kHsThreads) {
    const uint32_t kmin = mmk[2 * o], kmax = mmk[2 * o + 1];
    float* pp = a.part + ((int64_t)(model * a.G + grp) * 2) * a.B + b0 + o;
    pp[0] = kmin ? hs_unkey(~kmin) : __builtin_inff();
    pp[a.B] = kmax ? hs_unkey(kmax) : -__builtin_inff();
    if constexpr (MODE == HS_PRUNE) {
      const unsigned long long k = amk[o];
      a.argpos[(int64_t)(model * a.G + grp) * a.B + b0 + o] = k ? (int)~(uint32_t)k : -1;
    }
  }
  HS_STAMP_END();
}

// mm[model][0 / 1][b] = min / max over the G item groups' partials: a block
// of 256 threads takes 64 users of one model, 4 stripes of groups per user
// (8 loads in flight per thread), then folds the stripes in LDS.
__global__ __launch_bounds__(256) void hyb_mm_reduce_kernel(const float* __restrict__ part, int B, int G,
                                                           float* __restrict__ mm0, float* __restrict__ mm1) {
  __shared__ float slo[4][64], shi[4][64];
  const int bl = threadIdx.x & 63, st = threadIdx.x >> 6, model = blockIdx.y;
  const int b = blockIdx.x * 64 + bl;
  float lo = __builtin_inff(), hi = -__builtin_inff();
  if (b < B) {
    const float* p = part + (int64_t)model * G * 2 * B + b;
    for (int q0 = st; q0 < G; q0 += 4 * 8) {
      float l[8], h[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int q = q0 + 4 * e;
        l[e] = q < G ? p[(int64_t)q * 2 * B] : __builtin_inff();
        h[e] = q < G ? p[(int64_t)q * 2 * B + B] : -__builtin_inff();
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        lo = fminf(lo, l[e]);
        hi = fmaxf(hi, h[e]);
      }
    }
  }
  slo[st][bl] = lo;
  shi[st][bl] = hi;
  __syncthreads();
  if (st == 0 && b < B) {
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      lo = fminf(lo, slo[q][bl]);
      hi = fmaxf(hi, shi[q][bl]);
    }
    float* mm = model ? mm1 : mm0;
    mm[b] = lo;
    mm[B + b] = hi;
  }
}

int hs_slice_tiles(int dk) { return dk == 64 ? HsShape<64>::NI : (dk == 128 ? HsShape<128>::NI : HsShape<256>::NI); }

int hs_groups(int64_t n_items) {
  const int64_t g = (n_items + 255) / 256;
  return (int)(g < 128 ? (g < 1 ? 1 : g) : 128);
}

template <int DK>
static int hs_user_tile(int B) {
  constexpr int CU = 16 * HsShape<DK>::NU;
  int ub_max = kHsMaxUserBytes / HsShape<DK>::kRowB;
  ub_max = ub_max / CU * CU;
  if (ub_max > 4 * CU) ub_max = 4 * CU;  // <= 4 chunks (NCH instantiations)
  const int n_ut = (B + ub_max - 1) / ub_max;
  int UB = (B + n_ut - 1) / n_ut;
  return (UB + CU - 1) / CU * CU;
}

template <int DK, int NCH, int MODE>
static int hs_launch_n(HybScoresArgs& a, size_t lds, hipStream_t s) {
  const auto kfn = hyb_scores_kernel<DK, NCH, MODE>;
  if (!allow_max_lds(kfn))
    return check_launch("hyb_scores_kernel: LDS attribute");
  const int models = MODE == HS_FILTER ? 1 : 2;
  const int per_group = MODE == HS_FILTER ? a.fsplit : 1;
  hipLaunchKernelGGL(kfn, dim3((unsigned)(models * a.n_ut * a.G * per_group)), dim3(kHsThreads), lds, s, a);
  return check_launch("hyb_scores_kernel");
}

template <int DK, int MODE>
static int hs_launch(HybScoresArgs& a, float* mm0, float* mm1, hipStream_t s) {
  constexpr int CU = 16 * HsShape<DK>::NU;
  a.UB = hs_user_tile<DK>(a.B);
  a.n_ut = (a.B + a.UB - 1) / a.UB;
  size_t lds = (size_t)a.UB * HsShape<DK>::kRowB + (size_t)a.UB * (MODE == HS_PRUNE ? 16 : 8);
  if (MODE == HS_FILTER) {  // the rest of the 160 KiB stages survivors (12 B each)
    const size_t head = hs_filter_head(a.UB, HsShape<DK>::kRowB);
    a.sbuf = head < kHsMaxLds ? (int)((kHsMaxLds - head) / 12) : 0;
    if (a.sbuf > 8192) a.sbuf = 8192;
    lds = head + (size_t)a.sbuf * 12;
    // one model: split each item group over enough blocks to fill the CUs
    static const int cus = [] {
      int dev = 0, n = 256;
      if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
      return n > 0 ? n : 256;
    }();
    const int64_t slices = ((a.N + a.G - 1) / a.G + 16 * HsShape<DK>::NI - 1) / (16 * HsShape<DK>::NI);
    int fs = (cus + a.n_ut * a.G - 1) / (a.n_ut * a.G);
    if (fs > slices / 8) fs = (int)(slices / 8);  // >= one round of the 8 waves per block
    a.fsplit = fs < 1 ? 1 : fs;
  }
  int rc;
  switch (a.UB / CU) {
    case 1: rc = hs_launch_n<DK, 1, MODE>(a, lds, s); break;
    case 2: rc = hs_launch_n<DK, 2, MODE>(a, lds, s); break;
    case 3: rc = hs_launch_n<DK, 3, MODE>(a, lds, s); break;
    default: rc = hs_launch_n<DK, 4, MODE>(a, lds, s); break;
  }
  if (rc || MODE == HS_FILTER || mm0 == nullptr) return rc;  // no extremes wanted: the caller folds the partials
  hipLaunchKernelGGL(hyb_mm_reduce_kernel, dim3((unsigned)((a.B + 63) / 64), 2), dim3(256), 0, s, a.part, a.B, a.G,
                     mm0, mm1);
  return check_launch("hyb_mm_reduce_kernel");
}

template <int MODE>
static int hs_dispatch(HybScoresArgs& a, int dk, float* mm0, float* mm1, hipStream_t s) {
  switch (dk) {
    case 64: return hs_launch<64, MODE>(a, mm0, mm1, s);
    case 128: return hs_launch<128, MODE>(a, mm0, mm1, s);
    default: return hs_launch<256, MODE>(a, mm0, mm1, s);
  }
}

// The launch behind hrec_hybrid_scores and the pruned hybrid top-k
// (csrc/hybrid_prune.hip; arguments validated by the caller, n_items > 0).
int hybrid_scores_run(int mode, const float* als_users, int64_t als_ld, const int64_t* als_rows, int64_t n_als_rows,
                      int als_width, const float* tt_users, int64_t tt_ld, int tt_width, int n_users,
                      const void* als_items, const void* tt_items, int64_t n_items, int dk, float* als_out,
                      float* tt_out, int64_t ld_out, float* als_mm, float* tt_mm, float* part, int* argpos,
                      hipStream_t s, const uint16_t* uop, const HsFilter* filt) {
  HybScoresArgs a{};
  a.uop = uop;
  if (filt) {
    a.theta = filt->theta;
    a.hm = filt->hm;
    a.cap = filt->cap;
    a.cv = filt->cv;
    a.ci = filt->ci;
    a.cn = filt->cn;
  }
  a.users[0] = als_users;
  a.users[1] = tt_users;
  a.ld[0] = als_ld;
  a.ld[1] = tt_ld;
  a.rows[0] = als_rows;
  a.rows[1] = nullptr;
  a.n_rows[0] = als_rows ? n_als_rows : (int64_t)n_users;
  a.n_rows[1] = n_users;
  a.width[0] = als_width;
  a.width[1] = tt_width;
  a.B = n_users;
  a.items[0] = static_cast<const char*>(als_items);
  a.items[1] = static_cast<const char*>(tt_items);
  a.N = n_items;
  a.out[0] = als_out;
  a.out[1] = tt_out;
  a.ldo = ld_out;
  a.part = part;
  a.argpos = argpos;
  a.G = hs_groups(n_items);
  switch (mode) {
    case HS_PRUNE: return hs_dispatch<HS_PRUNE>(a, dk, als_mm, tt_mm, s);
    case HS_FILTER: return hs_dispatch<HS_FILTER>(a, dk, als_mm, tt_mm, s);
    default: return hs_dispatch<HS_FULL>(a, dk, als_mm, tt_mm, s);
  }
}

}  // namespace hrec

using namespace hrec;

#ifdef HREC_HS_STAMPS
extern "C" int hrec_debug_hs_stamps(unsigned long long* host_out, int reset) {
  (void)reset;
  if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_hs_stamps), sizeof(g_hs_stamps)) != hipSuccess) return -2;
  return 0;
}
#endif

extern "C" size_t hrec_hybrid_scores_workspace_bytes(int n_users, int64_t n_items) {
  const size_t B = (size_t)(n_users > 0 ? n_users : 0);
  return (size_t)2 * hs_groups(n_items) * 2 * B * sizeof(float) + 256;
}

extern "C" int hrec_hybrid_scores(const float* als_users, int64_t als_ld, const int64_t* als_rows,
                                  int64_t n_als_rows, int als_width,
                                  const float* tt_users, int64_t tt_ld, int tt_width, int n_users,
                                  const void* als_items, const void* tt_items, int64_t n_items, int dk,
                                  float* als_out, float* tt_out, int64_t ld_out, float* als_mm, float* tt_mm,
                                  void* workspace, size_t workspace_bytes, void* stream) {
  HREC_REQUIRE(dk == 64 || dk == 128 || dk == 256, "hybrid_scores: dk must be 64, 128 or 256 (got %d)", dk);
  HREC_REQUIRE(n_users >= 0 && n_items >= 0, "hybrid_scores: negative size");
  HREC_REQUIRE(n_items < 0x7fffffffll, "hybrid_scores: n_items must be < 2^31 - 1");
  HREC_REQUIRE(n_users <= (1 << 20), "hybrid_scores: at most 2^20 users per call");
  HREC_REQUIRE(als_width >= 0 && als_width <= dk && tt_width >= 0 && tt_width <= dk,
               "hybrid_scores: user widths must be in [0, dk]");
  HREC_REQUIRE(als_ld >= als_width && tt_ld >= tt_width, "hybrid_scores: row stride below the width");
  HREC_REQUIRE(n_als_rows >= 0, "hybrid_scores: negative n_als_rows");
  HREC_REQUIRE(ld_out >= n_items, "hybrid_scores: ld_out < n_items");
  if (n_users == 0) return HREC_OK;
  HREC_REQUIRE(als_mm && tt_mm && workspace, "hybrid_scores: null min/max output or workspace");
  HREC_REQUIRE(n_items == 0 || (als_users && tt_users && als_items && tt_items && als_out && tt_out),
               "hybrid_scores: null pointer");
  HREC_REQUIRE(((uintptr_t)als_items & 15) == 0 && ((uintptr_t)tt_items & 15) == 0,
               "hybrid_scores: item operands must be 16-B aligned");
  const size_t need = hrec_hybrid_scores_workspace_bytes(n_users, n_items);
  HREC_REQUIRE(workspace_bytes >= need, "hybrid_scores: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t s = as_stream(stream);
  if (n_items == 0) {  // no scores: min = +inf, max = -inf (hrec_rows_minmax_f32 of an empty row)
    hipLaunchKernelGGL(hyb_mm_reduce_kernel, dim3((unsigned)((n_users + 63) / 64), 2), dim3(256), 0, s,
                       static_cast<const float*>(workspace), n_users, 0, als_mm, tt_mm);
    return check_launch("hyb_mm_reduce_kernel");
  }
  return hybrid_scores_run(HS_FULL, als_users, als_ld, als_rows, n_als_rows, als_width, tt_users, tt_ld, tt_width,
                           n_users, als_items, tt_items, n_items, dk, als_out, tt_out, ld_out, als_mm, tt_mm,
                           static_cast<float*>(workspace), nullptr, s);
}
