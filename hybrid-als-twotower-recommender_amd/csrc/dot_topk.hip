// K8: user x item dot-product scoring on the matrix cores, with a fused top-k
// survivor filter — the "scored user-item pairs" half of the metric at
// BASELINE configs c4 (two-tower d = 128, 50M candidates) and c5 (bf16
// factors, d = 256).
//
// Replaces the two-tower scoring of the reference — Keras Dot(axes=1) over
// every candidate in model.predict (src/two_tower_model.py:80, :136-146) —
// and the ranking that follows it (sorted(..., reverse=True)[:k],
// src/hybrid_system.py:108; src/evaluation.py ranks the same way). The item
// tower output is computed once (hrec_tt_item_forward), so scoring is a GEMM
// [users, d] x [d, items] whose result is never written to HBM: every tile
// is compared in registers with a per-user lower bound of the k-th best
// score, and only survivors are appended to a per-user candidate list, which
// an exact stable top-k then ranks (ties -> smaller item index = the order
// of the reference's candidate list, which Python's stable sort keeps).
//
// Tiling (gfx950): a 512-thread block owns 128 users x 256 items; wave w
// computes 64 users (w & 1) x 64 items (w >> 1) as 4 x 4 tiles of 16 x 16.
// Every lane fetches 16 B per operand fragment: for bf16 that is one
// v_mfma_f32_16x16x32_bf16 operand (8 consecutive k), for f32 the operands of
// four v_mfma_f32_16x16x4_f32 steps (k = 16s + 4g + e, g = lane >> 4). The
// block's user rows sit in LDS (rows padded by 16 B: conflict-free b128
// reads); item fragments are loaded straight from HBM (each item is read by
// the 2 user-waves of its column; the user tiles of one item group run on the
// same XCD, so the other user tiles hit that XCD's L2).
#include <float.h>

#include <type_traits>

#include "common.h"

namespace hrec {

typedef float dot_f4 __attribute__((ext_vector_type(4)));
typedef __bf16 dot_bf8 __attribute__((ext_vector_type(8)));

constexpr int kDotThreads = 512;

template <bool BF16, int DK>
struct DotShape {
  static constexpr int kElem = BF16 ? 2 : 4;
  static constexpr int kStep = BF16 ? 32 : 16;     // k per 16-B lane fragment (over the 4 lane groups)
  static constexpr int kSteps = DK / kStep;
  static constexpr int kChunks = DK * kElem / 16;   // 16-B chunks per row
  static constexpr int kRow = DK * kElem + 16;      // LDS bytes per user row
};

typedef int dot_rsrc __attribute__((ext_vector_type(4)));
// buffer_load_dwordx4 ... idxen offen (structured: vindex * stride + voffset)
__device__ dot_f4 dot_sbuf_load(dot_rsrc rsrc, int vindex, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.struct.buffer.load.v4f32");

union DotFrag {
  int4 i;
  dot_f4 f;
};

template <bool BF16>
__device__ __forceinline__ void dot_mma(const DotFrag& a, const DotFrag& b, dot_f4& acc) {
  if constexpr (BF16) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(dot_bf8, a.i), __builtin_bit_cast(dot_bf8, b.i),
                                                  acc, 0, 0, 0);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.f[e], b.f[e], acc, 0, 0, 0);
  }
}

// FILTER = false: out[b * ldo + j] = score of item row j * item_step (j < n_items).
// FILTER = true:  append (score, j + idx_offset) to user b's candidate list when
//                 score >= thr[b * thr_stride] (a NaN threshold admits every score).
// Wave grid WU (users) x 8/WU (items); each wave owns NU x NI tiles of 16 x 16:
// a block covers 16 NU WU users x 16 NI (8/WU) items.
template <int NU_, int NI_, int WU_>
struct DotTiling {
  static constexpr int NU = NU_, NI = NI_, WU = WU_, WI = 8 / WU_;
  static constexpr int kUsers = 16 * NU * WU;
  static constexpr int kItems = 16 * NI * WI;
};

template <bool BF16, int DK, bool FILTER, class TL>
__global__ __launch_bounds__(kDotThreads) void dot_tile_kernel(
    const char* __restrict__ U, int B, const char* __restrict__ V, int64_t n_rows, int64_t n_items,
    int64_t item_step, int n_ut, float* __restrict__ out, int64_t ldo, const float* __restrict__ thr, int thr_stride,
    int cap, float* __restrict__ cand_v, int64_t* __restrict__ cand_i, int* __restrict__ cand_n, int64_t idx_offset) {
  using S = DotShape<BF16, DK>;
  constexpr int NU = TL::NU, NI = TL::NI;
  // User rows in LDS. Rows of >= 16 chunks of 16 B are XOR-swizzled (chunk q
  // of row r at q ^ (r & 15)): the 16 lanes of every ds_read_b128 lane group
  // then hit 16 distinct bank quads; shorter rows are padded by 16 B.
  constexpr bool kSwz = S::kChunks >= 16;
  constexpr int kRowB = kSwz ? S::kChunks * 16 : S::kRow;
  __shared__ __attribute__((aligned(16))) char us[TL::kUsers * kRowB];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int wu = w % TL::WU, wi = w / TL::WU;
  // XCD-aware map (blocks go round-robin over the 8 XCDs): XCD x takes the
  // consecutive logical blocks [x * nblk/8, (x+1) * nblk/8), user tile fastest.
  const int per_xcd = gridDim.x >> 3;
  const int lin = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  const int ut = lin % n_ut;
  const int64_t ig = lin / n_ut, n_ig = gridDim.x / n_ut;
  const int64_t n_it = (n_items + TL::kItems - 1) / TL::kItems;
  if (ig >= n_it) return;  // block-uniform
  const int b0 = ut * TL::kUsers;
  for (int o = threadIdx.x; o < TL::kUsers * S::kChunks; o += kDotThreads) {
    const int r = o / S::kChunks, q = o % S::kChunks;
    int4 v = {0, 0, 0, 0};
    if (b0 + r < B) v = *reinterpret_cast<const int4*>(U + (int64_t)(b0 + r) * (DK * S::kElem) + 16 * q);
    *reinterpret_cast<int4*>(us + r * kRowB + 16 * (kSwz ? q ^ (r & 15) : q)) = v;
  }
  // MFMA roles: A = items (output rows), B = users (output columns), so the
  // C/D layout puts ONE user on each lane per user tile: user ub + 16 u,
  // items j0 + 16 t + 4 g + r.
  const int ub = b0 + 16 * NU * wu + c;
  float th[FILTER ? NU : 1];  // NaN = absent user (never passes), -inf = admit every score
  if constexpr (FILTER) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int b = ub + 16 * u;
      float t = __builtin_nanf("");
      if (b < B) {
        t = thr[(int64_t)b * thr_stride];
        t = t == t ? t : -INFINITY;
      }
      th[u] = t;
    }
  }
  __syncthreads();
  const char* ubase = us + (16 * NU * wu + c) * kRowB;
  const int xq = c ^ g;  // swizzled chunk of step ks: (4 ks + g) ^ c = 4 ks ^ (c ^ g)
  auto user_frag = [&](int u, int ks) {
    DotFrag a;
    const int off = kSwz ? 16 * ((4 * ks) ^ xq) : 64 * ks + 16 * g;
    a.i = *reinterpret_cast<const int4*>(ubase + 16 * u * kRowB + off);
    return a;
  };
  // Item fragments: structured buffer loads (address = V + vindex * row
  // bytes + 16 g; the hardware range check returns zeros for vindex >=
  // n_rows, so tails need no clamping), flowing through a ring of P steps
  // issued P steps ahead across tile boundaries (the next tile's first steps
  // load during the current tile's last MFMAs). User fragments are read one
  // step ahead from LDS (the last step of a tile reads step 0 again: users
  // do not change between tiles).
  constexpr int PB = FILTER ? 4 : 2;
  constexpr int P = BF16 ? (S::kSteps < PB ? S::kSteps : PB) : (S::kSteps < 2 ? S::kSteps : 2);
  static_assert(S::kSteps % P == 0, "ring depth must divide the k steps");
  // one resource per item tile, based at the tile's first row (row indices
  // relative to it: a resource spans at most 4 GiB, see rows_rsrc)
  const int voff = 16 * g;
  auto rsrc_of = [&](int64_t tile) { return rows_rsrc(V, tile * TL::kItems * item_step, DK * S::kElem, n_rows); };
  auto rows_of = [&](int64_t tile, int (&vi)[NI]) {
    const int64_t jb = tile * TL::kItems + 16 * NI * wi;
#pragma unroll
    for (int t = 0; t < NI; ++t) {
      const int64_t j = jb + 16 * t + c;
      vi[t] = j < n_items ? (int)((j - tile * TL::kItems) * item_step) : 0x7fffffff;
    }
  };
  int vcur[NI], vnext[NI];
  rows_of(ig, vcur);
  dot_rsrc rs_cur = rsrc_of(ig), rs_next = rs_cur;
  DotFrag ring[P][NI];
#pragma unroll
  for (int q = 0; q < P; ++q)
#pragma unroll
    for (int t = 0; t < NI; ++t) ring[q][t].f = dot_sbuf_load(rs_cur, vcur[t], voff + 64 * q, 0, 0);
  DotFrag ua[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) ua[u] = user_frag(u, 0);
  for (int64_t it = ig; it < n_it; it += n_ig) {
    const int64_t j0 = it * TL::kItems + 16 * NI * wi;
    rows_of(it + n_ig, vnext);
    rs_next = rsrc_of(it + n_ig);
    dot_f4 acc[NU][NI];
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int t = 0; t < NI; ++t) acc[u][t] = dot_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int k0 = 0; k0 < S::kSteps; k0 += P) {  // P steps per trip: ring slots stay compile-time
#pragma unroll
      for (int q = 0; q < P; ++q) {
        const int ks = k0 + q;
        DotFrag b[NI], a[NU];
        const bool same = ks + P < S::kSteps;
        const int off = voff + 64 * (same ? ks + P : ks + P - S::kSteps);
#pragma unroll
        for (int t = 0; t < NI; ++t) {
          b[t] = ring[q][t];
          ring[q][t].f = dot_sbuf_load(same ? rs_cur : rs_next, same ? vcur[t] : vnext[t], off, 0, 0);
        }
        const int kn = ks + 1 < S::kSteps ? ks + 1 : 0;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          a[u] = ua[u];
          ua[u] = user_frag(u, kn);
        }
#pragma unroll
        for (int u = 0; u < NU; ++u)
#pragma unroll
          for (int t = 0; t < NI; ++t) dot_mma<BF16>(b[t], a[u], acc[u][t]);
        __builtin_amdgcn_sched_barrier(0);  // keep each step's prefetches in its step (VGPR budget)
      }
    }
#pragma unroll
    for (int t = 0; t < NI; ++t) vcur[t] = vnext[t];
    rs_cur = rs_next;
    if constexpr (!FILTER) {
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int b = ub + 16 * u;
        if (b >= B) continue;
        float* o = out + (int64_t)b * ldo;
#pragma unroll
        for (int t = 0; t < NI; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int64_t j = j0 + 16 * t + 4 * g + r;
            if (j < n_items) o[j] = acc[u][t][r];
          }
      }
    } else {
      // Fast path: one v_cmp per score into a wave mask; survivors are rare,
      // so the append path below runs for few tiles. Items past n_items
      // (zero fragments) are rejected there.
      uint64_t any = 0;
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        float mx = acc[u][0][0];
#pragma unroll
        for (int t = 0; t < NI; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (t || r) mx = fmaxf(mx, acc[u][t][r]);
        any |= __ballot(mx >= th[u]);
      }
      if (any) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int b = ub + 16 * u;
#pragma unroll
          for (int t = 0; t < NI; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int64_t j = j0 + 16 * t + 4 * g + r;
              const float sc = acc[u][t][r];
              if (j < n_items && sc >= th[u]) {
                const int pos = atomicAdd(&cand_n[b], 1);
                if (pos < cap) {
                  cand_v[(int64_t)b * cap + pos] = sc;
                  cand_i[(int64_t)b * cap + pos] = j + idx_offset;
                }
              }
            }
        }
      }
    }
  }
}

__global__ void dot_overflow_kernel(const int* __restrict__ cand_n, int n_users, int cap, int* __restrict__ flag) {
  for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < n_users; b += gridDim.x * blockDim.x)
    if (cand_n[b] > cap) atomicOr(flag, 1);
}

__global__ void dot_offset_kernel(int64_t* __restrict__ idx, int64_t n, int64_t off) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n && idx[i] >= 0) idx[i] += off;
}

// f32 -> bf16 bit patterns, round to nearest even (NaN stays NaN).
__global__ void f32_to_bf16_kernel(const float* __restrict__ in, int64_t n, uint16_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t x = __float_as_uint(in[i]);
    uint16_t h;
    if ((x & 0x7fffffffu) > 0x7f800000u) h = (uint16_t)((x >> 16) | 0x40);
    else h = (uint16_t)((x + 0x7fffu + ((x >> 16) & 1u)) >> 16);
    out[i] = h;
  }
}

// Resident-users variant: the block keeps UB users (up to 128 KB of LDS) and
// every wave keeps its 32 items' fragments for the whole d in registers while
// it sweeps all UB users in chunks of 128 — an item fragment is fetched from
// L2 once per UB users instead of once per 128 (the L2 re-reads and misses
// of the 128-user tiling were the stall). During the last chunk each item
// fragment is refilled with the next tile's as soon as its step has used it
// the last time, so the loads have a whole chunk plus a step to land.
#ifndef HREC_RES_NU
#define HREC_RES_NU 4
#endif
constexpr int kResUserBytes = 128 * 1024;
constexpr size_t kMaxLds = 160 * 1024;  // per workgroup (allow_max_lds raises the default)
constexpr int kResNU = HREC_RES_NU;  // user tiles per chunk (64 users): leaves VGPRs for the prefetches
#ifndef HREC_RES_NI_BF16
#define HREC_RES_NI_BF16 4
#endif
constexpr int kResNIbf16 = HREC_RES_NI_BF16;  // item tiles per wave, bf16 at d <= 128 (2 or 4)

template <bool BF16, int DK, bool FILTER, int NI_>
__global__ __launch_bounds__(kDotThreads) void dot_res_kernel(
    const char* __restrict__ U, int B, int UB, const char* __restrict__ V, int64_t n_rows, int64_t n_items,
    int64_t item_step, int n_ut, float* __restrict__ out, int64_t ldo, const float* __restrict__ thr, int thr_stride,
    int64_t thr_per, int cap, float* __restrict__ cand_v, int64_t* __restrict__ cand_i, int* __restrict__ cand_n,
    int64_t idx_offset, int sbuf, int inf_none) {
  using S = DotShape<BF16, DK>;
  // NI = 4: 32-user chunks (8 MFMAs per 2 user-fragment reads, as 4 x 4
  // would be, at the register budget of two waves per SIMD)
  constexpr int NI = NI_, NU = NI_ == 4 ? 2 : kResNU, KS = S::kSteps;
  constexpr int CU = 16 * NU;  // users per chunk
  constexpr int kItems = 8 * 16 * NI;  // per block tile
  constexpr bool kSwz = S::kChunks >= 16;
  constexpr int kRowB = kSwz ? S::kChunks * 16 : S::kRow;
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  char* us = dsm;                                      // UB user rows
  float* ths = reinterpret_cast<float*>(dsm + (size_t)UB * kRowB);  // UB thresholds
  // FILTER: survivors are staged in LDS and appended once per tile (below)
  int* cnt_l = reinterpret_cast<int*>(ths + UB);                  // [UB] per-user counts, then list bases
  int* ovf_l = cnt_l + UB;                                          // [UB] survivors dropped (buffer full)
  // entries staged per tile: three counters in rotation (tile i uses i % 3;
  // its flush resets the one of tile i + 2), so a tile without survivors
  // needs a single barrier
  int* bn = ovf_l + UB;
  // [sbuf] survivor meta (user << 22 | item in tile << 12 | list offset), then [sbuf] scores
  uint32_t* buf = reinterpret_cast<uint32_t*>(dsm + (((size_t)UB * kRowB + (size_t)UB * 12 + 12 + 15) & ~(size_t)15));
  float* buf_s = reinterpret_cast<float*>(buf + sbuf);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int per_xcd = gridDim.x >> 3;
  const int lin = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  const int ut = lin % n_ut;
  const int64_t ig = lin / n_ut, n_ig = gridDim.x / n_ut;
  const int64_t n_it = (n_items + kItems - 1) / kItems;
  if (ig >= n_it) return;  // block-uniform
  const int b0 = ut * UB;
  // batches of 8 independent 16-B loads per thread in flight
  for (int o0 = threadIdx.x; o0 < UB * S::kChunks; o0 += 8 * kDotThreads) {
    int4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = o0 + j * kDotThreads;
      const int r = o / S::kChunks, q = o % S::kChunks;
      v[j] = int4{0, 0, 0, 0};
      if (o < UB * S::kChunks && b0 + r < B)
        v[j] = *reinterpret_cast<const int4*>(U + (int64_t)(b0 + r) * (DK * S::kElem) + 16 * q);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = o0 + j * kDotThreads;
      const int r = o / S::kChunks, q = o % S::kChunks;
      if (o < UB * S::kChunks) *reinterpret_cast<int4*>(us + r * kRowB + 16 * (kSwz ? q ^ (r & 15) : q)) = v[j];
    }
  }
  if (FILTER) {
    for (int o = threadIdx.x; o < UB; o += kDotThreads) {
      if (thr_per == 0) {
        float t = __builtin_nanf("");  // absent user: never passes
        if (b0 + o < B) {
          t = thr[(int64_t)(b0 + o) * thr_stride];
          // NaN admits all; +inf admits scores >= +inf, or none (inf_none:
          // the pruned hybrid's dead users, whose chunks are then skipped)
          t = t == t ? (inf_none && t == INFINITY ? __builtin_nanf("") : t) : -INFINITY;
        }
        ths[o] = t;
      }
      cnt_l[o] = 0;
      ovf_l[o] = 0;
    }
    if (threadIdx.x < 3) bn[threadIdx.x] = 0;
  }
  __syncthreads();
  const int xq = c ^ g;
  // one resource per item tile, based at the tile's first row (rows_rsrc)
  const int voff = 16 * g;
  auto rsrc_of = [&](int64_t tile) { return rows_rsrc(V, tile * kItems * item_step, DK * S::kElem, n_rows); };
  auto rows_of = [&](int64_t tile, int (&vi)[NI]) {
    const int64_t jb = tile * kItems + 16 * NI * w;
#pragma unroll
    for (int t = 0; t < NI; ++t) {
      const int64_t j = jb + 16 * t + c;
      vi[t] = (tile < n_it && j < n_items) ? (int)((j - tile * kItems) * item_step) : 0x7fffffff;
    }
  };
  int vnext[NI];
  rows_of(ig, vnext);
  dot_rsrc rsrc = rsrc_of(ig);
  DotFrag it_f[KS][NI];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int t = 0; t < NI; ++t) it_f[ks][t].f = dot_sbuf_load(rsrc, vnext[t], voff + 64 * ks, 0, 0);
  const int n_ch = (UB + 16 * NU - 1) / (16 * NU);
  DotFrag ua[NU];  // user fragments of the next step (chunk 0, step 0 first)
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int off = kSwz ? 16 * xq : 16 * g;
    ua[u].i = *reinterpret_cast<const int4*>(us + (16 * u + c) * kRowB + off);
  }
  int cur = 0;  // FILTER: this tile's staging counter
  for (int64_t it = ig; it < n_it; it += n_ig, cur = cur == 2 ? 0 : cur + 1) {
    const int64_t j0 = it * kItems + 16 * NI * w;
    // the wave's valid items (positions relative to its first item, 32-bit)
    const int w_n = (int)(n_items - j0 < 16 * NI ? (n_items - j0 > 0 ? n_items - j0 : 0) : 16 * NI);
    if (FILTER && thr_per > 0) {
      // per-group bounds: each user's loosest bound over the tile's groups
      // gates the ballot (the survivor pass compares each item exactly)
      const int64_t q0 = it * kItems / thr_per;
      const int64_t q1 = ((it + 1) * kItems < n_items ? (it + 1) * kItems : n_items) - 1;
      for (int o = threadIdx.x; o < UB; o += kDotThreads) {
        float t = __builtin_nanf("");
        if (b0 + o < B) {
          const float* tr = thr + (int64_t)(b0 + o) * thr_stride;
          t = INFINITY;
          for (int64_t gq = q0; gq <= q1 / thr_per; ++gq) {
            const float x = tr[gq];
            t = fminf(t, x == x ? x : -INFINITY);
          }
          if (inf_none && t == INFINITY) t = __builtin_nanf("");  // every group dead: the chunks skip this user
        }
        ths[o] = t;
      }
      __syncthreads();
    }
    rows_of(it + n_ig, vnext);
    rsrc = rsrc_of(it + n_ig);  // the last chunk refills the fragments with the next tile's
    auto user_frag = [&](int ch, int u, int ks) {
      DotFrag a;
      const int off = kSwz ? 16 * ((4 * ks) ^ xq) : 64 * ks + 16 * g;
      a.i = *reinterpret_cast<const int4*>(us + (CU * ch + 16 * u + c) * kRowB + off);
      return a;
    };
    // The last chunk is peeled (compile-time LAST): its item refills are then
    // unconditional, so the waitcnt pass can count them instead of draining.
    auto chunk = [&](int ch, auto last_t) {
      constexpr bool last = decltype(last_t)::value;
      // the next chunk's first user fragments load during this chunk's last
      // step (after the last chunk: chunk 0 again, for the next tile)
      const int ch_next = ch + 1 < n_ch ? ch + 1 : 0;
      dot_f4 acc[NU][NI];
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int t = 0; t < NI; ++t) acc[u][t] = dot_f4{0.f, 0.f, 0.f, 0.f};
      // this chunk's bounds (LDS), read before the MFMAs: per user, or
      // (thr_per > 0) the user's loosest bound over the tile's groups — the
      // flush then checks each staged item against its own group's bound
      float th[NU];
      if constexpr (FILTER) {
        bool live = false;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          th[u] = CU * ch + 16 * u + c < UB ? ths[CU * ch + 16 * u + c] : __builtin_nanf("");
          live = live || th[u] == th[u];
        }
        if (__ballot(live) == 0) {
          // no user of the chunk can have a survivor in the tile (NaN bounds:
          // absent users, +inf bounds): skip its MFMAs, keep the pipelines
          // (the next chunk's first user fragments; the next tile's items)
#pragma unroll
          for (int u = 0; u < NU; ++u) ua[u] = user_frag(ch_next, u, 0);
          if constexpr (last) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#pragma unroll
              for (int t = 0; t < NI; ++t) it_f[ks][t].f = dot_sbuf_load(rsrc, vnext[t], voff + 64 * ks, 0, 0);
          }
          return;
        }
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        DotFrag a[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          a[u] = ua[u];
          ua[u] = ks + 1 < KS ? user_frag(ch, u, ks + 1) : user_frag(ch_next, u, 0);
        }
#pragma unroll
        for (int u = 0; u < NU; ++u)
#pragma unroll
          for (int t = 0; t < NI; ++t) dot_mma<BF16>(it_f[ks][t], a[u], acc[u][t]);
        if constexpr (last) {  // step ks of this tile is done: refill it with the next tile's
#pragma unroll
          for (int t = 0; t < NI; ++t) it_f[ks][t].f = dot_sbuf_load(rsrc, vnext[t], voff + 64 * ks, 0, 0);
        }
        // Order the step: each next-step user read sits between MFMA pairs, so
        // the LDS reads overlap the whole step instead of trailing it.
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
          __builtin_amdgcn_sched_group_barrier(0x008, NI, 0);  // MFMA
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // C/D: lane holds user (CU ch + 16 u + c), items j0 + 16 t + 4 g + r
      if constexpr (!FILTER) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int b = b0 + CU * ch + 16 * u + c;
          if (b >= B || CU * ch + 16 * u + c >= UB) continue;
          float* o = out + (int64_t)b * ldo;
#pragma unroll
          for (int t = 0; t < NI; ++t) {
            const int64_t j = j0 + 16 * t + 4 * g;
            if (j + 3 < n_items && (ldo & 3) == 0) {
              *reinterpret_cast<float4*>(o + j) = make_float4(acc[u][t][0], acc[u][t][1], acc[u][t][2], acc[u][t][3]);
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (j + r < n_items) o[j + r] = acc[u][t][r];
            }
          }
        }
      } else {
        // one compare per user tile: the lane's max over its 8 items (fmaxf
        // drops NaN scores, which never pass anyway; a NaN bound never passes)
        uint64_t any = 0;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          float mx = acc[u][0][0];
#pragma unroll
          for (int t = 0; t < NI; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (t || r) mx = fmaxf(mx, acc[u][t][r]);
          any |= __ballot(mx >= th[u]);
        }
        if (any) {
          // Survivors -> the block's LDS staging buffer (one LDS reservation
          // per lane); no global atomic waits in the MFMA loop. Entry: user
          // << 22 | item in tile << 12 (| the user-list offset, set at the
          // flush) + the score.
          uint32_t msk[NU];
          int cnt = 0;
#pragma unroll
          for (int u = 0; u < NU; ++u) {
            uint32_t m = 0;
#pragma unroll
            for (int t = 0; t < NI; ++t)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (16 * t + 4 * g + r < w_n && acc[u][t][r] >= th[u]) m |= 1u << (4 * t + r);
            msk[u] = m;
            cnt += __popc(m);
          }
          int pos = cnt ? atomicAdd(&bn[cur], cnt) : 0;  // LDS: the lanes' reservations serialise in the LDS unit only
          const int jt = 16 * NI * w;  // the wave's first item in the tile
#pragma unroll
          for (int u = 0; u < NU; ++u) {
            if (msk[u] == 0) continue;
            const int ul = CU * ch + 16 * u + c;
#pragma unroll
            for (int t = 0; t < NI; ++t)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if ((msk[u] >> (4 * t + r)) & 1u) {
                  const float sc = acc[u][t][r];
                  if (pos < sbuf) {
                    buf[pos] = ((uint32_t)ul << 22) | ((uint32_t)(jt + 16 * t + 4 * g + r) << 12);
                    buf_s[pos] = sc;
                  } else {
                    ovf_l[ul] = 1;  // buffer full: handled at the flush
                  }
                  ++pos;
                }
          }
        }
      }
    };
    for (int ch = 0; ch + 1 < n_ch; ++ch) chunk(ch, std::false_type{});
    chunk(n_ch - 1, std::true_type{});
    if constexpr (FILTER) {
      // flush the tile's staged survivors: per-user offsets (LDS atomics),
      // one list reservation per user (global atomics, all in flight), then
      // the appends
      __syncthreads();
      const int nb = bn[cur] < sbuf ? bn[cur] : sbuf;  // block-uniform: bn[cur] changes no more this tile
      if (threadIdx.x == 0) bn[cur == 0 ? 2 : cur - 1] = 0;  // the counter of tile i + 2 (read by all at tile i - 1)
      if (nb == 0) continue;  // nothing staged: no list to extend
      for (int e = threadIdx.x; e < nb; e += kDotThreads) {
        const uint32_t x = buf[e];
        if (thr_per > 0) {  // the item's own group bound (the ballot used the tile's loosest)
          const int64_t j = it * kItems + (int64_t)((x >> 12) & 1023u);
          float t = thr[(int64_t)(b0 + (int)(x >> 22)) * thr_stride + j / thr_per];
          t = t == t ? t : -INFINITY;
          if (!(buf_s[e] >= t) || (inf_none && t == INFINITY)) {
            buf[e] = 0xffffffffu;  // dropped (no user 1023: UB <= 1023)
            continue;
          }
        }
        buf[e] = x | (uint32_t)atomicAdd(&cnt_l[x >> 22], 1);
      }
      __syncthreads();
      for (int o = threadIdx.x; o < UB; o += kDotThreads) {
        const int k = cnt_l[o];
        if (k > 0) cnt_l[o] = atomicAdd(&cand_n[b0 + o], k);
        if (ovf_l[o]) {
          // the staging buffer dropped survivors of this user: its list is
          // marked overflowing (cand_n > cap) and its free slots filled with
          // (-inf, INT64_MAX - 1), so every slot < cap holds an entry and the
          // list's k-th best stays a valid lower bound (hrec_dot_topk's
          // second round)
          const int64_t b = b0 + o;
          for (int p = atomicAdd(&cand_n[b], cap + 1); p < cap; ++p) {
            cand_v[b * cap + p] = -INFINITY;
            cand_i[b * cap + p] = INT64_MAX - 1;
          }
          ovf_l[o] = 0;
        }
      }
      __syncthreads();
      for (int e = threadIdx.x; e < nb; e += kDotThreads) {
        const uint32_t x = buf[e];
        if (x == 0xffffffffu) continue;
        const int ul = (int)(x >> 22);
        const int p = cnt_l[ul] + (int)(x & 4095u);
        if (p < cap) {
          const int64_t b = b0 + ul;
          cand_v[b * cap + p] = buf_s[e];
          cand_i[b * cap + p] = it * kItems + (int64_t)((x >> 12) & 1023u) + idx_offset;
        }
      }
      __syncthreads();
      for (int o = threadIdx.x; o < UB; o += kDotThreads) cnt_l[o] = 0;
      __syncthreads();
    }
  }
}

// Tilings of the tile kernel (f32 at dk 256): FILTER passes keep each item
// fragment for 128 users (item bytes through the vector cache halve vs 64 x 64
// wave tiles; the user fragments come from LDS, which has twice the bandwidth).
typedef DotTiling<4, 4, 2> DotTileA;   // 128 users x 256 items, wave 64 x 64
typedef DotTiling<8, 2, 1> DotTileB;   // 128 users x 256 items, wave 128 x 32

// Grid of the tile kernel: 8 * n_ut * m blocks (a multiple of 8 so the XCD map
// is a bijection), about two 512-thread blocks per CU, no more item groups
// than item tiles.
// blocks_per_cu: what the block's LDS allows (the resident-user kernel with
// > 80 KB: one, so a second round of blocks would re-stage every user row).
static unsigned dot_grid(int n_ut, int64_t n_items, int tile_items, int blocks_per_cu = 2) {
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  const int64_t n_it = (n_items + tile_items - 1) / tile_items;
  const int64_t target = (int64_t)cus * blocks_per_cu;
  int64_t m = (target + 8 * n_ut - 1) / (8 * n_ut);
  const int64_t m_max = (n_it + 7) / 8;
  if (m > m_max) m = m_max;
  if (m < 1) m = 1;
  return (unsigned)(8 * n_ut * m);
}

template <bool FILTER, class TL>
static int dot_launch_t(const void* U, int B, const void* V, int64_t n_rows, int64_t n_items, int64_t step, int dk,
                        int bf16, float* out, int64_t ldo, const float* thr, int thr_stride, int cap, float* cv,
                        int64_t* ci, int* cn, int64_t off, hipStream_t s) {
  const int n_ut = (B + TL::kUsers - 1) / TL::kUsers;
  const dim3 grid(dot_grid(n_ut, n_items, TL::kItems)), block(kDotThreads);
  const char* u = (const char*)U;
  const char* v = (const char*)V;
#define HREC_DOT(BF, DK)                                                                                         \
  hipLaunchKernelGGL((dot_tile_kernel<BF, DK, FILTER, TL>), grid, block, 0, s, u, B, v, n_rows, n_items, step, n_ut, \
                     out, ldo, thr, thr_stride, cap, cv, ci, cn, off)
  if (bf16) {
    switch (dk) {
      case 32: HREC_DOT(true, 32); break;
      case 64: HREC_DOT(true, 64); break;
      case 128: HREC_DOT(true, 128); break;
      default: HREC_DOT(true, 256); break;
    }
  } else {
    switch (dk) {
      case 32: HREC_DOT(false, 32); break;
      case 64: HREC_DOT(false, 64); break;
      case 128: HREC_DOT(false, 128); break;
      default: HREC_DOT(false, 256); break;
    }
  }
#undef HREC_DOT
  return check_launch("dot_tile_kernel");
}

template <bool BF16, int DK, bool FILTER>
static auto dot_res_pick(int ni) {
  if constexpr (BF16 && DK <= 128) {
    if (ni == 4) return dot_res_kernel<BF16, DK, FILTER, 4>;
  }
  return dot_res_kernel<BF16, DK, FILTER, 2>;
}

template <bool FILTER>
static int dot_launch_res(const void* U, int B, const void* V, int64_t n_rows, int64_t n_items, int64_t step, int dk,
                          int bf16, float* out, int64_t ldo, const float* thr, int thr_stride, int cap, float* cv,
                          int64_t* ci, int* cn, int64_t off, hipStream_t s, int64_t thr_per = 0,
                          int inf_none = 0, int ub_cap = 0) {
  const int row_b = dk * (bf16 ? 2 : 4);
  const int row_lds = row_b >= 256 ? row_b : row_b + 16;
  int ub_max = kResUserBytes / row_lds;
  if (ub_cap > 0 && ub_max > ub_cap) ub_max = ub_cap;  // more user tiles: more blocks for a short item range
  ub_max = ub_max / (16 * kResNU) * (16 * kResNU);
  if (ub_max < 16 * kResNU) ub_max = 16 * kResNU;
  const int n_ut = (B + ub_max - 1) / ub_max;
  int UB = (B + n_ut - 1) / n_ut;
  UB = (UB + 16 * kResNU - 1) / (16 * kResNU) * (16 * kResNU);
  // FILTER: + per-user counts, the staging counter and a survivor buffer in
  // the rest of the 160 KiB (at most 4096 entries: 12-bit offsets)
  size_t lds = (size_t)UB * row_lds + (size_t)UB * 4;
  int sbuf = 0;
  if (FILTER) {
    const size_t head = ((size_t)UB * row_lds + (size_t)UB * 12 + 12 + 15) & ~(size_t)15;
    const size_t room = head < kMaxLds ? (kMaxLds - head) / 8 : 0;
    sbuf = (int)(room < 4096 ? room : 4096);
    lds = head + (size_t)sbuf * 8;
  }
  // bf16 at d <= 128: 64 items per wave (4 item tiles), so each user fragment
  // read from LDS feeds 4 MFMAs instead of 2 (the LDS read chain, not the
  // matrix cores, was what the waves waited on); f32 and d = 256 keep 32
  const int ni = (bf16 && dk <= 128) ? kResNIbf16 : 2;
  const dim3 grid(dot_grid(n_ut, n_items, 128 * ni, lds > kMaxLds / 2 ? 1 : 2)), block(kDotThreads);
  const char* u = (const char*)U;
  const char* v = (const char*)V;
#define HREC_DOTR(BF, DK)                                                                                      \
  do {                                                                                                         \
    auto kfn = dot_res_pick<BF, DK, FILTER>(ni);                                                               \
    if (!allow_max_lds(kfn))                                                                                   \
      return check_launch("dot_res_kernel: LDS attribute");                                                   \
    hipLaunchKernelGGL(kfn, grid, block, lds, s, u, B, UB, v, n_rows, n_items, step, n_ut, out, ldo, thr,         \
                       thr_stride, thr_per, cap, cv, ci, cn, off, sbuf, inf_none);                             \
  } while (0)
  if (bf16) {
    switch (dk) {
      case 32: HREC_DOTR(true, 32); break;
      case 64: HREC_DOTR(true, 64); break;
      case 128: HREC_DOTR(true, 128); break;
      default: HREC_DOTR(true, 256); break;
    }
  } else {
    switch (dk) {
      case 32: HREC_DOTR(false, 32); break;
      case 64: HREC_DOTR(false, 64); break;
      default: HREC_DOTR(false, 128); break;
    }
  }
#undef HREC_DOTR
  return check_launch("dot_res_kernel");
}

template <bool FILTER>
static int dot_launch(const void* U, int B, const void* V, int64_t n_rows, int64_t n_items, int64_t step, int dk,
                      int bf16, float* out, int64_t ldo, const float* thr, int thr_stride, int cap, float* cv,
                      int64_t* ci, int* cn, int64_t off, hipStream_t s) {
  if (dot_gemv_applies(B, step, dk, bf16))  // a few users: the streaming GEMV kernel (csrc/dot_gemv.hip)
    return dot_gemv_run<FILTER>(U, B, V, n_rows, n_items, step, dk, bf16, out, ldo, thr, thr_stride, cap, cv, ci, cn,
                                off, s);
  if (bf16 || dk <= 128)  // the resident-user kernel
    return dot_launch_res<FILTER>(U, B, V, n_rows, n_items, step, dk, bf16, out, ldo, thr, thr_stride, cap, cv, ci,
                                  cn, off, s);
  // f32 at dk 256 (the resident users would not fit the LDS): the tile kernel
  if constexpr (!FILTER) {
    return dot_launch_t<false, DotTileA>(U, B, V, n_rows, n_items, step, dk, bf16, out, ldo, thr, thr_stride, cap,
                                         cv, ci, cn, off, s);
  }
  return dot_launch_t<FILTER, DotTileB>(U, B, V, n_rows, n_items, step, dk, bf16, out, ldo, thr, thr_stride, cap, cv,
                                        ci, cn, off, s);
}

// Sample size and candidate capacity of the threshold filter: the k-th best
// of S strided items is a lower bound of the k-th best of all n items, and
// about k * n / S items beat it, so S = 4 k n / cap leaves ~4x headroom.
static int64_t dot_cap(int kk) { return kk <= 64 ? 8192 : 128 * (int64_t)kk; }
static int64_t dot_sample(int64_t n, int kk) {
  if (n <= 16384) return n;
  int64_t s = (4 * (int64_t)kk * n + dot_cap(kk) - 1) / dot_cap(kk);
  if (s < 8192) s = 8192;
  return s < n ? s : n;
}

// The survivor filter alone (the pruned hybrid's pass 2, csrc/hybrid_prune.hip):
// append (score, j) of every item j with score >= thr[b * thr_stride + j /
// thr_per] to user b's list (cap entries; cn[b] counts every survivor, so
// cn[b] > cap = overflow). Always the resident-user kernel (the only one with
// per-group bounds). Here a +inf bound admits nothing (a dead group / user,
// skipped); hrec_dot_topk's filter keeps +inf meaning "score >= +inf".
int dot_filter_run(const void* U, int B, const void* V, int64_t n_items, int dk, int bf16, const float* thr,
                   int thr_stride, int64_t thr_per, int cap, float* cv, int64_t* ci, int* cn, hipStream_t s) {
  if (!bf16 && dk > 128) {
    set_error("dot_filter_run: f32 operands need dk <= 128");
    return HREC_E_INVALID;
  }
  return dot_launch_res<true>(U, B, V, n_items, n_items, 1, dk, bf16, nullptr, 0, thr, thr_stride, cap, cv, ci, cn, 0,
                              s, thr_per, 1);
}

// Scores of the resident-user kernel with at most ub_cap users per block
// (the pruned ALS top-k's sample: 8192 items are too few tiles to fill the
// chip with the full 128 KiB of resident users).
int dot_scores_run(const void* U, int B, const void* V, int64_t n_items, int dk, int bf16, float* out, int64_t ldo,
                   hipStream_t s, int ub_cap) {
  if (!bf16 && dk > 128) {
    set_error("dot_scores_run: f32 operands need dk <= 128");
    return HREC_E_INVALID;
  }
  return dot_launch_res<false>(U, B, V, n_items, n_items, 1, dk, bf16, out, ldo, nullptr, 0, 0, nullptr, nullptr,
                               nullptr, 0, s, 0, 0, ub_cap);
}

int count_overflow(const int* cn, int n_users, int cap, int* flag, hipStream_t s) {
  hipLaunchKernelGGL(dot_overflow_kernel, dim3(64), dim3(256), 0, s, cn, n_users, cap, flag);
  return check_launch("dot_overflow_kernel");
}

int offset_ids(int64_t* idx, int64_t n, int64_t off, hipStream_t s) {
  if (n <= 0 || off == 0) return HREC_OK;
  hipLaunchKernelGGL(dot_offset_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, idx, n, off);
  return check_launch("dot_offset_kernel");
}

static char* dot_carve(char*& p, size_t bytes) {
  char* r = p;
  p += (bytes + 255) & ~(size_t)255;
  return r;
}

}  // namespace hrec

using namespace hrec;

static int dot_check(const void* U, int B, const void* V, int64_t n_items, int dk, int dtype, const char* who) {
  HREC_REQUIRE(dk == 32 || dk == 64 || dk == 128 || dk == 256, "%s: dk must be 32, 64, 128 or 256 (got %d)", who, dk);
  HREC_REQUIRE(dtype == 0 || dtype == 1, "%s: dtype must be 0 (f32) or 1 (bf16)", who);
  HREC_REQUIRE(B >= 0 && n_items >= 0, "%s: negative size", who);
  HREC_REQUIRE(B <= (1 << 24), "%s: at most 2^24 users per call", who);
  HREC_REQUIRE(n_items < 0x7fffffffll, "%s: n_items must be < 2^31 - 1", who);
  HREC_REQUIRE(B == 0 || n_items == 0 || (U && V), "%s: null pointer", who);
  HREC_REQUIRE(((uintptr_t)U & 15) == 0 && ((uintptr_t)V & 15) == 0, "%s: vectors must be 16-B aligned", who);
  return HREC_OK;
}

extern "C" int hrec_f32_to_bf16(const float* in, int64_t n, uint16_t* out, void* stream) {
  HREC_REQUIRE(n >= 0, "f32_to_bf16: negative size");
  if (n == 0) return HREC_OK;
  HREC_REQUIRE(in && out, "f32_to_bf16: null pointer");
  int64_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), in, n, out);
  return check_launch("f32_to_bf16_kernel");
}

extern "C" int hrec_dot_scores(const void* user_vec, int n_users, const void* item_vec, int64_t n_items, int dk,
                               int dtype, float* out, int64_t ld_out, void* stream) {
  int rc = dot_check(user_vec, n_users, item_vec, n_items, dk, dtype, "dot_scores");
  if (rc) return rc;
  HREC_REQUIRE(ld_out >= n_items, "dot_scores: ld_out < n_items");
  if (n_users == 0 || n_items == 0) return HREC_OK;
  HREC_REQUIRE(out, "dot_scores: null output");
  return dot_launch<false>(user_vec, n_users, item_vec, n_items, n_items, 1, dk, dtype, out, ld_out, nullptr, 0, 0, nullptr,
                           nullptr, nullptr, 0, as_stream(stream));
}

extern "C" int hrec_dot_filter(const void* user_vec, int n_users, const void* item_vec, int64_t n_items, int dk,
                               int dtype, const float* thr, int thr_stride, int64_t thr_per, int cap, float* cand_val,
                               int64_t* cand_idx, int* cand_n, void* stream) {
  int rc = dot_check(user_vec, n_users, item_vec, n_items, dk, dtype, "dot_filter");
  if (rc) return rc;
  HREC_REQUIRE(dtype == 1 || dk <= 128, "dot_filter: f32 operands need dk <= 128");
  HREC_REQUIRE(cap >= 0 && thr_per >= 0 && thr_stride >= 0, "dot_filter: bad cap / bound layout");
  HREC_REQUIRE(thr_per == 0 || thr_stride >= (n_items + thr_per - 1) / thr_per,
               "dot_filter: thr_stride < the number of item groups");
  if (n_users == 0 || n_items == 0) return HREC_OK;
  HREC_REQUIRE(thr && cand_n && (cap == 0 || (cand_val && cand_idx)), "dot_filter: null pointer");
  return dot_filter_run(user_vec, n_users, item_vec, n_items, dk, dtype, thr, thr_stride, thr_per, cap, cand_val,
                        cand_idx, cand_n, as_stream(stream));
}

extern "C" size_t hrec_dot_topk_workspace_bytes(int n_users, int64_t n_items, int top_k) {
  const size_t B = (size_t)(n_users > 0 ? n_users : 0);
  const int kk = (int)(top_k < n_items ? top_k : n_items);
  if (kk <= 0) return 256;
  const int64_t S = dot_sample(n_items, kk), cap = dot_cap(kk);
  size_t b = B * (size_t)S * 4 + 256;                 // sample scores
  b += topk_ws_bytes(B, S, kk, 4) + 256;               // sample top-k workspace
  b += B * (size_t)kk * 12 + 512;                      // sample top-k values / indices
  b += B * (size_t)cap * 12 + 512;                     // candidates
  b += B * 4 + 256;                                    // counters
  b += topk_ws_bytes(B, cap, kk, 4) + 256;             // final top-k workspace
  return b;
}

extern "C" int hrec_dot_topk(const void* user_vec, int n_users, const void* item_vec, int64_t n_items, int dk,
                             int dtype, int top_k, const float* thr_in, int64_t idx_offset, int64_t* out_idx,
                             float* out_val, int* overflow, void* workspace, size_t workspace_bytes, void* stream) {
  int rc = dot_check(user_vec, n_users, item_vec, n_items, dk, dtype, "dot_topk");
  if (rc) return rc;
  HREC_REQUIRE(top_k >= 1 && top_k <= 1024, "dot_topk: top_k must be in [1, 1024]");
  HREC_REQUIRE(n_users < 65536, "dot_topk: at most 65535 users per call");
  if (n_users == 0 || n_items == 0) return HREC_OK;
  HREC_REQUIRE(out_idx && out_val && overflow && workspace, "dot_topk: null pointer");
  const size_t need = hrec_dot_topk_workspace_bytes(n_users, n_items, top_k);
  HREC_REQUIRE(workspace_bytes >= need, "dot_topk: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t s = as_stream(stream);
  const int kk = (int)(top_k < n_items ? top_k : n_items);
  const int64_t S = dot_sample(n_items, kk), cap = dot_cap(kk);
  char* p = (char*)workspace;
  float* samp = (float*)dot_carve(p, (size_t)n_users * S * 4);
  char* tws = dot_carve(p, topk_ws_bytes(n_users, S, kk, 4));
  float* sv = (float*)dot_carve(p, (size_t)n_users * kk * 4);
  int64_t* si = (int64_t*)dot_carve(p, (size_t)n_users * kk * 8);
  float* cv = (float*)dot_carve(p, (size_t)n_users * cap * 4);
  int64_t* ci = (int64_t*)dot_carve(p, (size_t)n_users * cap * 8);
  int* cn = (int*)dot_carve(p, (size_t)n_users * 4);
  char* fws = dot_carve(p, topk_ws_bytes(n_users, cap, kk, 4));
  if (hipMemsetAsync(overflow, 0, sizeof(int), s) != hipSuccess) return check_launch("dot_topk: memset");
  if (S == n_items && thr_in == nullptr) {  // small: every score, exact top-k
    rc = dot_launch<false>(user_vec, n_users, item_vec, n_items, n_items, 1, dk, dtype, samp, n_items, nullptr, 0, 0, nullptr,
                           nullptr, nullptr, 0, s);
    if (rc) return rc;
    rc = topk_rows<float>(samp, n_users, n_items, n_items, kk, out_idx, out_val, tws, (size_t)1 << 62, s);
  } else {
    const float* thr = thr_in;
    int thr_stride = 1;
    if (thr == nullptr) {  // 1) thresholds: the kk-th best of S strided items
      const int64_t step = n_items / S;
      rc = dot_launch<false>(user_vec, n_users, item_vec, n_items, S, step, dk, dtype, samp, S, nullptr, 0, 0, nullptr,
                             nullptr, nullptr, 0, s);
      if (rc) return rc;
      rc = topk_rows<float>(samp, n_users, S, S, kk, si, sv, tws, (size_t)1 << 62, s);
      if (rc) return rc;
      thr = sv + (kk - 1);
      thr_stride = kk;
    }
    // 2) fused score + survivor filter over every item
    if (hipMemsetAsync(cn, 0, (size_t)n_users * 4, s) != hipSuccess)
      return check_launch("dot_topk: memset");
    rc = dot_launch<true>(user_vec, n_users, item_vec, n_items, n_items, 1, dk, dtype, nullptr, 0, thr, thr_stride, (int)cap,
                          cv, ci, cn, 0, s);
    if (rc) return rc;
    hipLaunchKernelGGL(dot_overflow_kernel, dim3(64), dim3(256), 0, s, cn, n_users, (int)cap, overflow);
    rc = check_launch("dot_overflow_kernel");
    if (rc) return rc;
    // 3) exact stable top-k of the survivors (item index breaks ties)
    rc = topk_rows<float>(cv, n_users, cap, cap, kk, out_idx, out_val, fws, (size_t)1 << 62, s, ci, cn);
  }
  if (rc) return rc;
  return offset_ids(out_idx, (int64_t)n_users * kk, idx_offset, s);
}
