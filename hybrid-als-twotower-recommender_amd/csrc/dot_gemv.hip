// K8v: dot-product scoring of a FEW users (B <= 4) against every item — the
// reference's own call shape: one user ranked against all candidates
// (TwoTowerModel.predict_for_user, src/two_tower_model.py:136-146, Keras Dot
// over every candidate row; the hybrid's per-user call, src/hybrid_system.py
// :95-116). With one user the work is a GEMV: 2 flops per 4 B of item
// operand, so the kernel is bound by streaming the [N, dk] item matrix from
// HBM once, and the MFMA tile kernel (16 users per tile, 15 of them empty)
// has nothing to offer it.
//
// Layout: a row of dk elements is R = dk * elem bytes = L chunks of 16 B. A
// wave reads 64 rows as L loads; load t covers G = 64 / L consecutive rows
// (lane = g * L + c reads chunk c of row t * G + g), so every load instruction
// of the wave is one contiguous G * R = 1 KiB span and the wave's L loads one
// contiguous span of 64 rows (64 R bytes: 32 KiB at d = 128 f32). Each lane keeps the
// partial dot of its chunk for each of the L loads; a transpose reduction
// (log2 L butterfly steps, each lane keeping half of its values and adding
// the partner's other half) leaves lane (g, c) with the full score of row
// c * G + g — 2 (L - 1) shuffles per 64 rows instead of L * log2 L.
//
// FILTER = false: out[b * ldo + j] = score of item row j * item_step.
// FILTER = true:  append (score, j + idx_offset) to user b's list when score
//                 >= thr[b * thr_stride] (NaN admits every score, +inf the
//                 scores >= +inf), one wave-aggregated atomic per user and
//                 wave; cand_n[b] counts every survivor (> cap = overflow).


#include "common.h"

namespace hrec {

constexpr int kGemvThreads = 256;
constexpr int kGemvMaxB = 4;

template <bool BF16, int DK>
struct GemvShape {
  static constexpr int kElem = BF16 ? 2 : 4;
  static constexpr int R = DK * kElem;  // row bytes
  static constexpr int L = R / 16;      // lanes per row (one 16-B chunk each)
  static constexpr int G = 64 / L;      // rows per wave load
  static constexpr int E = 16 / kElem;  // elements per chunk
  static_assert(L >= 1 && L <= 64 && (L & (L - 1)) == 0, "row must be 16 B .. 1 KiB, a power of two");
};

// 16 B of the operand as E f32 values (bf16: exact widening).
template <bool BF16>
__device__ __forceinline__ void gemv_unpack(const int4 v, float* x) {
  if constexpr (BF16) {
    const uint32_t w[4] = {(uint32_t)v.x, (uint32_t)v.y, (uint32_t)v.z, (uint32_t)v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      x[2 * q] = __uint_as_float(w[q] << 16);
      x[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
    }
  } else {
    x[0] = __int_as_float(v.x);
    x[1] = __int_as_float(v.y);
    x[2] = __int_as_float(v.z);
    x[3] = __int_as_float(v.w);
  }
}

// 4 waves per SIMD (<= 128 registers): a wave's loads are issued in batches
// of kGemvBatch (16 B each per lane), so 16 waves per CU keep ~128 KiB of
// the operand in flight — well past what the CU's share of HBM bandwidth
// needs to cover the memory latency.
#ifndef HREC_GEMV_BATCH
#define HREC_GEMV_BATCH 8
#endif
#ifndef HREC_GEMV_WAVES
#define HREC_GEMV_WAVES 4
#endif
#ifndef HREC_GEMV_AUX
#define HREC_GEMV_AUX 2  // cache-policy bits of the item loads: non-temporal (the operand streams once)
#endif
constexpr int kGemvBatch = HREC_GEMV_BATCH;

typedef int gemv_v4i __attribute__((ext_vector_type(4)));
// buffer_load_dwordx4 ... offen (raw: base + voffset, range-checked in bytes:
// loads past num_records return zeros)
__device__ gemv_v4i gemv_raw_load(hrec_rsrc_t rsrc, uint32_t voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.raw.buffer.load.v4i32");

// Raw (unstructured) buffer resource over [base, base + bytes), bytes clamped
// to the 32-bit range.
__device__ __forceinline__ hrec_rsrc_t gemv_rsrc(const char* base, int64_t bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t n = bytes <= 0 ? 0u : (bytes >= 0xffffffffll ? 0xffffffffu : (uint32_t)bytes);
  hrec_rsrc_t r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  r.z = __builtin_amdgcn_readfirstlane((int)n);
  r.w = 0x00020000;
  return r;
}

template <bool BF16, int DK, int NB, bool FILTER>
__global__ __launch_bounds__(kGemvThreads, HREC_GEMV_WAVES) void dot_gemv_kernel(
    const char* __restrict__ U, int B, const char* __restrict__ V, int64_t n_rows, int64_t n_items,
    int64_t item_step, float* __restrict__ out, int64_t ldo, const float* __restrict__ thr, int thr_stride, int cap,
    float* __restrict__ cand_v, int64_t* __restrict__ cand_i, int* __restrict__ cand_n, int64_t idx_offset) {
#pragma clang fp contract(off)
  using S = GemvShape<BF16, DK>;
  constexpr int L = S::L, G = S::G, E = S::E;
  const int lane = threadIdx.x & 63;
  const int c = lane % L, g = lane / L;
  // this lane's chunk of every user (absent users: zeros, never reported)
  float u[NB][E];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    int4 v = {0, 0, 0, 0};
    if (b < B) v = *reinterpret_cast<const int4*>(U + (int64_t)b * S::R + 16 * c);
    gemv_unpack<BF16>(v, u[b]);
  }
  float th[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    th[b] = __builtin_nanf("");  // absent user: nothing passes
    if (FILTER && b < B) {
      const float t = thr[(int64_t)b * thr_stride];
      th[b] = t == t ? t : -INFINITY;  // NaN bound admits every score
    }
  }
  const int64_t n_tiles = (n_items + 63) / 64;
  const int64_t nw = (int64_t)gridDim.x * (kGemvThreads / 64);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // lane offset inside a tile and the step between loads (the host keeps a
  // tile's 64 rows x step x R below 2^32)
  const uint32_t lane_off = (uint32_t)g * (uint32_t)(item_step * S::R) + 16u * (uint32_t)c;
  const uint32_t load_step = (uint32_t)(G * item_step * S::R);
  const int64_t v_bytes = n_rows * S::R;
  for (int64_t tile = (int64_t)blockIdx.x * (kGemvThreads / 64) + wave; tile < n_tiles; tile += nw) {
    const int64_t j0 = tile * 64;
    // one resource per tile, based at its first row: rows past the matrix
    // read as zeros (their scores are never reported)
    const int64_t row0_b = j0 * item_step * S::R;
    const hrec_rsrc_t rs = gemv_rsrc(V + row0_b, v_bytes - row0_b);
    float p[NB][L];
    // the L loads in batches, each batch's partial dots (one per load and
    // user) as its data lands
    constexpr int T = L < kGemvBatch ? L : kGemvBatch;
#pragma unroll
    for (int t0 = 0; t0 < L; t0 += T) {
      gemv_v4i raw[T];
#pragma unroll
      for (int q = 0; q < T; ++q) raw[q] = gemv_raw_load(rs, lane_off + (uint32_t)(t0 + q) * load_step, 0, HREC_GEMV_AUX);
#pragma unroll
      for (int q = 0; q < T; ++q) {
        float x[E];
        gemv_unpack<BF16>(int4{raw[q].x, raw[q].y, raw[q].z, raw[q].w}, x);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          float a = u[b][0] * x[0];
#pragma unroll
          for (int e = 1; e < E; ++e) a = __builtin_fmaf(u[b][e], x[e], a);
          p[b][t0 + q] = a;
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // one batch's loads live at a time (VGPR budget)
    }
    // transpose reduction over the L lanes of each row group: at offset h the
    // lane keeps the half of its 2h values whose index bit h equals its own
    // chunk bit h and adds the partner's copy of that half
#pragma unroll
    for (int h = L / 2; h >= 1; h >>= 1) {
      const bool hi = (c & h) != 0;
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < h; ++i) {
          const float keep = hi ? p[b][i + h] : p[b][i];
          const float send = hi ? p[b][i] : p[b][i + h];
          p[b][i] = keep + __shfl_xor(send, h, 64);
        }
    }
    // lane (g, c) now holds the scores of row j = j0 + c G + g
    const int64_t j = j0 + c * G + g;
    const bool ok = j < n_items;
    if constexpr (!FILTER) {
      if (ok) {
#pragma unroll
        for (int b = 0; b < NB; ++b)
          if (b < B) out[(int64_t)b * ldo + j] = p[b][0];
      }
    } else {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const bool pass = ok && p[b][0] >= th[b];
        const uint64_t m = __ballot(pass);
        if (m == 0) continue;  // wave-uniform
        const int leader = __ffsll((long long)m) - 1;
        int base = 0;
        if (lane == leader) base = atomicAdd(&cand_n[b], __popcll(m));
        base = __shfl(base, leader, 64);
        if (pass) {
          const int pos =
              base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          if (pos < cap) {
            cand_v[(int64_t)b * cap + pos] = p[b][0];
            cand_i[(int64_t)b * cap + pos] = j + idx_offset;
          }
        }
      }
    }
  }
}

template <bool BF16, int DK, int NB, bool FILTER>
static int gemv_launch_t(const void* U, int B, const void* V, int64_t n_rows, int64_t n_items, int64_t step, float* out, int64_t ldo,
                         const float* thr, int thr_stride, int cap, float* cv, int64_t* ci, int* cn, int64_t off,
                         hipStream_t s) {
  auto kfn = dot_gemv_kernel<BF16, DK, NB, FILTER>;
  // a grid of what is resident at once: each wave strides over the 64-row tiles
  static const int resident = [kfn] {
    int dev = 0, cus = 256, per = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kfn, kGemvThreads, 0) != hipSuccess || per < 1) per = 2;
    return (cus > 0 ? cus : 256) * per;
  }();
  const int64_t tiles = (n_items + 63) / 64;
  int64_t blocks = (tiles + kGemvThreads / 64 - 1) / (kGemvThreads / 64);
  if (blocks > resident) blocks = resident;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(kfn, dim3((unsigned)blocks), dim3(kGemvThreads), 0, s, (const char*)U, B, (const char*)V,
                     n_rows, n_items, step, out, ldo, thr, thr_stride, cap, cv, ci, cn, off);
  return check_launch("dot_gemv_kernel");
}

// users per launch for B users (1, 2 or 4: absent ones are zero rows)
static int gemv_nb(int B) { return B <= 1 ? 1 : (B == 2 ? 2 : 4); }

// NB x L partial dots per lane stay in registers at 4 waves per SIMD only up
// to 32 of them (64 spill): wider rows / more users take the matrix-core path
template <bool BF16, int DK, int NB>
constexpr bool gemv_fits() {
  return NB * GemvShape<BF16, DK>::L <= 32;
}

template <bool BF16, int DK, bool FILTER>
static int gemv_launch_nb(const void* U, int B, const void* V, int64_t n_rows, int64_t n_items, int64_t step,
                          float* out, int64_t ldo, const float* thr, int thr_stride, int cap, float* cv, int64_t* ci,
                          int* cn, int64_t off, hipStream_t s) {
#define HREC_GEMV_NB(NB)                                                                                         \
  if constexpr (gemv_fits<BF16, DK, NB>()) {                                                                     \
    if (gemv_nb(B) == NB)                                                                                        \
      return gemv_launch_t<BF16, DK, NB, FILTER>(U, B, V, n_rows, n_items, step, out, ldo, thr, thr_stride, cap,  \
                                                 cv, ci, cn, off, s);                                            \
  }
  HREC_GEMV_NB(1)
  HREC_GEMV_NB(2)
  HREC_GEMV_NB(4)
#undef HREC_GEMV_NB
  set_error("dot_gemv: %d users at dk %d do not fit the kernel", B, DK);
  return HREC_E_INVALID;
}

static bool gemv_fits_rt(int nb, int dk, int bf16) {
  const int L = dk * (bf16 ? 2 : 4) / 16;
  return nb * L <= 32;
}

// Measured on the c4 one-user call (50M x 128, scripts/gpu_gemv_ab.sh): f32
// 6.15 ms on the matrix cores (16x16x4 f32 tiles, 15 of 16 users empty) ->
// 3.95 ms here (non-temporal loads; 4.35 cached); bf16 2.23 ms on the matrix
// cores vs 2.29-2.59 here, so bf16 operands keep the matrix-core path.
bool dot_gemv_applies(int B, int64_t step, int dk, int bf16) {
  if (bf16) return false;  // bf16 operands keep the matrix-core path (measured faster)
  // a tile's 64 rows x step must stay within one 32-bit buffer offset
  const int64_t tile_bytes = 64 * step * (int64_t)dk * 4;
  return B >= 1 && B <= kGemvMaxB && gemv_fits_rt(gemv_nb(B), dk, 0) && tile_bytes < ((int64_t)1 << 32);
}

template <bool FILTER>
int dot_gemv_run(const void* U, int B, const void* V, int64_t n_rows, int64_t n_items, int64_t step, int dk, int bf16, float* out,
                 int64_t ldo, const float* thr, int thr_stride, int cap, float* cv, int64_t* ci, int* cn, int64_t off,
                 hipStream_t s) {
#define HREC_GEMV(BF, DK) \
  return gemv_launch_nb<BF, DK, FILTER>(U, B, V, n_rows, n_items, step, out, ldo, thr, thr_stride, cap, cv, ci, cn, off, s)
  if (bf16) {
    set_error("dot_gemv_run: f32 operands only (dot_gemv_applies)");
    return HREC_E_INVALID;
  }
  switch (dk) {
    case 32: HREC_GEMV(false, 32);
    case 64: HREC_GEMV(false, 64);
    case 128: HREC_GEMV(false, 128);
    default: HREC_GEMV(false, 256);
  }
#undef HREC_GEMV
}

template int dot_gemv_run<false>(const void*, int, const void*, int64_t, int64_t, int64_t, int, int, float*, int64_t,
                                 const float*, int, int, float*, int64_t*, int*, int64_t, hipStream_t);
template int dot_gemv_run<true>(const void*, int, const void*, int64_t, int64_t, int64_t, int, int, float*, int64_t,
                                const float*, int, int, float*, int64_t*, int*, int64_t, hipStream_t);

}  // namespace hrec
