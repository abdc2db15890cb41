// K8v: dot-product scoring of a FEW users (B <= 4, f32 operands) against every
// item — the reference's own call shape: one user ranked against all
// candidates (TwoTowerModel.predict_for_user, src/two_tower_model.py:136-146,
// Keras Dot over every candidate row; the hybrid's per-user call,
// src/hybrid_system.py:95-116). With one user the work is a GEMV: 2 flops per
// 4 B of item operand, so the kernel is bound by streaming the [N, dk] item
// matrix from HBM once.
//
// Same bits as the matrix-core tiles of >= 5 users (csrc/dot_topk.hip): the
// scores are the SAME v_mfma_f32_16x16x4_f32 sequence — per score, k steps of
// 16 (k = 16 ks + 4 g + e: instruction e of step ks takes the four lane
// groups' component e), accumulator starting at zero — so a user's score bits
// do not depend on how many users share the call (a one-user
// hybrid call and a batched recommender must rank near-ties alike). The
// matrix cores are mostly idle here (one user column of 16 in use), but at
// dk/64 MFMAs of 32 cycles per item per SIMD they still outrun HBM by ~2.5x
// at dk = 128 (dk = 256: ~2.5x as well, at half the items per byte).
//
// Layout: the MFMA A operand is 16 items (rows) x 4 k: lane (g, c) = lane
// (lane >> 4, lane & 15) holds item row c's 16-B chunk at byte 64 ks + 16 g,
// one structured buffer load per (tile, ks) — 16 rows x 64 contiguous bytes
// per wave load, every byte of a row read once per call; the B operand is the
// users: lane (g, c) holds user c's same chunk (zeros for c >= B). A wave owns
// NT = 8 / KS tiles of 16 items at a time (NT x KS x 16 B = 128 B of item
// operand per lane), the next round's loads issued before this round's MFMAs
// (two rounds in registers); the waves of a CU overlap each other's too.
//
// FILTER = false: out[b * ldo + j] = score of item row j * item_step.
// FILTER = true:  append (score, j + idx_offset) to user b's list when score
//                 >= thr[b * thr_stride] (NaN admits every score, +inf the
//                 scores >= +inf), one wave-aggregated atomic per user and
//                 (tile, register); cand_n[b] counts every survivor (> cap =
//                 overflow).
#include "common.h"

namespace hrec {

constexpr int kGemvThreads = 256;
constexpr int kGemvMaxB = 4;

typedef float gemv_f4 __attribute__((ext_vector_type(4)));

#ifndef HREC_GEMV_PIPE
// 1 = the next round's loads issued before this round's MFMAs (with half the
// tiles per round: the same registers). c4 one user, top-5 (50M x 128):
// 4.34 -> 4.23 ms; 50M x 64: 2.50 -> 2.25 ms; 25M x 256 unchanged (4.33)
#define HREC_GEMV_PIPE 1
#endif
#ifndef HREC_GEMV_NTDIV
#define HREC_GEMV_NTDIV 2  // item tiles per wave round / this (with PIPE: two rounds' loads in registers)
#endif
#ifndef HREC_GEMV_NTX
#define HREC_GEMV_NTX 1  // A/B builds: item tiles per wave round x this
#endif
template <int DK>
struct GemvShape {
  static constexpr int R = DK * 4;                  // row bytes (f32)
  static constexpr int KS = DK / 16;                // k steps of 16 (4 MFMAs each)
  static constexpr int NT0 = (KS >= 16 ? 1 : 16 / KS) * HREC_GEMV_NTX / HREC_GEMV_NTDIV;
  static constexpr int NT = NT0 < 1 ? 1 : NT0;  // 16-item tiles per wave round
  static constexpr int kItems = 16 * NT;            // items per wave round
};

__device__ gemv_f4 gemv_sbuf_load(hrec_rsrc_t rsrc, int vindex, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.struct.buffer.load.v4f32");

#ifndef HREC_GEMV_AUX
// cache-policy bits of the item loads: 0 = cached. A wave load covers 64 B of
// each of 16 rows, so the other half of every 128-B line arrives with the
// next k step's load and must still be in the L1; measured at c4 (50M x 128,
// one user, top-5): cached 4.38 ms, non-temporal (2) 4.69 ms; two 16-item
// tiles more per round (HREC_GEMV_NTX 2) 4.67 ms
#define HREC_GEMV_AUX 0
#endif

template <int DK, bool FILTER>
__global__ __launch_bounds__(kGemvThreads) void dot_gemv_kernel(
    const float* __restrict__ U, int B, const char* __restrict__ V, int64_t n_rows, int64_t n_items,
    int64_t item_step, float* __restrict__ out, int64_t ldo, const float* __restrict__ thr, int thr_stride, int cap,
    float* __restrict__ cand_v, int64_t* __restrict__ cand_i, int* __restrict__ cand_n, int64_t idx_offset) {
  using S = GemvShape<DK>;
  constexpr int KS = S::KS, NT = S::NT;
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, c = lane & 15;
  // the user operand of every k step (user c; absent users: zeros, never reported)
  gemv_f4 uf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    uf[ks] = gemv_f4{0.f, 0.f, 0.f, 0.f};
    if (c < B) uf[ks] = *reinterpret_cast<const gemv_f4*>(U + (int64_t)c * DK + 16 * ks + 4 * g);
  }
  float th = __builtin_nanf("");  // absent user: nothing passes
  if (FILTER && c < B) {
    const float t = thr[(int64_t)c * thr_stride];
    th = t == t ? t : -INFINITY;  // NaN bound admits every score
  }
  const int64_t n_rounds = (n_items + S::kItems - 1) / S::kItems;
  const int64_t nw = (int64_t)gridDim.x * (kGemvThreads / 64);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool vec = !FILTER && (ldo & 3) == 0 && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
  // one resource per round, based at its first row (rows past the matrix
  // read as zeros; their scores are never reported)
  auto load_round = [&](int64_t rd, gemv_f4 (&it)[NT][KS]) {
    const hrec_rsrc_t rs = rows_rsrc(V, rd * S::kItems * item_step, S::R, n_rows);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        it[t][ks] = gemv_sbuf_load(rs, (int)((16 * t + c) * item_step), 64 * ks + 16 * g, 0, HREC_GEMV_AUX);
  };
  int64_t rd = (int64_t)blockIdx.x * (kGemvThreads / 64) + wave;
#if HREC_GEMV_PIPE
  gemv_f4 nx[NT][KS];  // the next round's items, loading during this round's MFMAs
  if (rd < n_rounds) load_round(rd, nx);
#endif
  for (; rd < n_rounds; rd += nw) {
    const int64_t j0 = rd * S::kItems;
    gemv_f4 it[NT][KS];
#if HREC_GEMV_PIPE
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) it[t][ks] = nx[t][ks];
    if (rd + nw < n_rounds) load_round(rd + nw, nx);
#else
    load_round(rd, it);
#endif
    gemv_f4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = gemv_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(it[t][ks][e], uf[ks][e], acc[t], 0, 0, 0);
    // lane (g, c): user c, items j0 + 16 t + 4 g + r
    if constexpr (!FILTER) {
      if (c < B) {
        float* o = out + (int64_t)c * ldo;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int64_t j = j0 + 16 * t + 4 * g;
          if (vec && j + 3 < n_items) {
            *reinterpret_cast<gemv_f4*>(o + j) = acc[t];
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (j + r < n_items) o[j + r] = acc[t][r];
          }
        }
      }
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t j = j0 + 16 * t + 4 * g + r;
          const bool pass = c < B && j < n_items && acc[t][r] >= th;
          const uint64_t m = __ballot(pass);
          if (m == 0) continue;  // wave-uniform
          for (int b = 0; b < B; ++b) {
            const uint64_t mb = m & (0x0001000100010001ull << b);  // lanes (g, c = b)
            if (mb == 0) continue;
            const int leader = __builtin_ctzll(mb);
            int base = 0;
            if (lane == leader) base = atomicAdd(&cand_n[b], __popcll(mb));
            base = __shfl(base, leader, 64);
            if (pass && c == b) {
              const int pos = base + __popcll(mb & ((1ull << lane) - 1));
              if (pos < cap) {
                cand_v[(int64_t)b * cap + pos] = acc[t][r];
                cand_i[(int64_t)b * cap + pos] = j + idx_offset;
              }
            }
          }
        }
    }
  }
}

template <int DK, bool FILTER>
static int gemv_launch_t(const void* U, int B, const void* V, int64_t n_rows, int64_t n_items, int64_t step,
                         float* out, int64_t ldo, const float* thr, int thr_stride, int cap, float* cv, int64_t* ci,
                         int* cn, int64_t off, hipStream_t s) {
  auto kfn = dot_gemv_kernel<DK, FILTER>;
  // a grid of what is resident at once: each wave strides over the rounds
  static const int resident = [kfn] {
    int dev = 0, cus = 256, per = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kfn, kGemvThreads, 0) != hipSuccess || per < 1) per = 2;
    return (cus > 0 ? cus : 256) * per;
  }();
  const int64_t rounds = (n_items + GemvShape<DK>::kItems - 1) / GemvShape<DK>::kItems;
  int64_t blocks = (rounds + kGemvThreads / 64 - 1) / (kGemvThreads / 64);
  if (blocks > resident) blocks = resident;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(kfn, dim3((unsigned)blocks), dim3(kGemvThreads), 0, s, (const float*)U, B, (const char*)V,
                     n_rows, n_items, step, out, ldo, thr, thr_stride, cap, cv, ci, cn, off);
  return check_launch("dot_gemv_kernel");
}

// Measured on the c4 one-user call (50M x 128): bf16 operands keep the
// matrix-core tile path (2.23 ms against 2.29-2.59 for a streaming bf16 GEMV).
bool dot_gemv_applies(int B, int64_t step, int dk, int bf16) {
  if (bf16) return false;
  // a round's rows x step must stay within one 32-bit buffer offset (a round
  // is 16 KiB of rows at every dk: kItems * R = 16 NT * 4 dk)
  const int64_t round_bytes = (int64_t)16384 * HREC_GEMV_NTX * step;  // >= the real round (NTDIV shrinks it)
  return B >= 1 && B <= kGemvMaxB && (dk == 32 || dk == 64 || dk == 128 || dk == 256) &&
         round_bytes < ((int64_t)1 << 32);
}

template <bool FILTER>
int dot_gemv_run(const void* U, int B, const void* V, int64_t n_rows, int64_t n_items, int64_t step, int dk, int bf16,
                 float* out, int64_t ldo, const float* thr, int thr_stride, int cap, float* cv, int64_t* ci, int* cn,
                 int64_t off, hipStream_t s) {
  if (bf16 || B < 1 || B > kGemvMaxB) {
    set_error("dot_gemv_run: f32 operands and 1..4 users only (dot_gemv_applies)");
    return HREC_E_INVALID;
  }
#define HREC_GEMV(DK) \
  return gemv_launch_t<DK, FILTER>(U, B, V, n_rows, n_items, step, out, ldo, thr, thr_stride, cap, cv, ci, cn, off, s)
  switch (dk) {
    case 32: HREC_GEMV(32);
    case 64: HREC_GEMV(64);
    case 128: HREC_GEMV(128);
    default: HREC_GEMV(256);
  }
#undef HREC_GEMV
}

template int dot_gemv_run<false>(const void*, int, const void*, int64_t, int64_t, int64_t, int, int, float*, int64_t,
                                 const float*, int, int, float*, int64_t*, int*, int64_t, hipStream_t);
template int dot_gemv_run<true>(const void*, int, const void*, int64_t, int64_t, int64_t, int, int, float*, int64_t,
                                const float*, int, int, float*, int64_t*, int*, int64_t, hipStream_t);

}  // namespace hrec
