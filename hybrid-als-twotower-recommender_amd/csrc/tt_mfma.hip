// K4m: the Keras item tower of src/two_tower_model.py:38-66 on the f32
// matrix cores (v_mfma_f32_16x16x4_f32: an exact f32 fma chain per k-step,
// the arithmetic of Keras' f32 Dense):
//
//   h        = relu(numeric @ W1 + b1)              Dense(16, relu)   (:56-57)
//   z        = [E_item[i] | E_man[m] | E_cat[c] | h]   (d + 32)        (:60)
//   item_vec = LN(z @ W2 + b2)                      Dense(d) + LN     (:63-64)
//
// One wave owns 16 items x all dp = 16·NT output columns (NT accumulator
// tiles). The K axis (d + 32, padded per 16-column block) is walked one
// 16-wide block at a time; inside a block the k order is permuted so that
// every lane feeds 4 MFMA k-steps from ONE 16-B gather of its item's row:
// lane l loads z[row l%16][16·kb + 4·(l/16) .. +3] and k-step j uses
// component j — the B operand follows the same permutation. W2 sits in LDS,
// staged once per persistent workgroup in exactly that permuted order
// (quads XOR-swizzled by column so a ds_read_b128 of 16 lanes hits 16
// distinct bank quads); at dp = 256 (295 KB, more than the LDS) the B
// fragments are read from global memory (L2-resident).
// Epilogue in registers: + b2, LayerNormalization (Keras: epsilon 1e-3,
// biased variance, two-pass mean / variance) reduced over the 16 lanes that
// hold a row, y = xhat·gamma + beta; optional saves for the backward pass
// (z [n, d+32], xhat [n, d], 1/std [n]).
//
// Algorithmic work per item: 2·(d+32)·d flops; HBM bytes: one gathered
// E_item row (4d) + E_man/E_cat rows (64) + numeric (8) + ids (12) + the
// output row (4d).
#include <type_traits>

#include "common.h"

namespace hrec {

typedef float f4m __attribute__((ext_vector_type(4)));

#ifndef HREC_TT_FWD_ABLATE
#define HREC_TT_FWD_ABLATE 0  // timing-only builds: 1 = no LN epilogue, 2 = also no A gathers
#endif

constexpr float kLnEpsM = 1e-3f;

// compile-time loop: f(std::integral_constant<int, i>) for i in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

struct TTFwd {
  int d;
  const float *ie, *me, *ce, *w1, *b1, *w2, *b2, *g, *be;
};

// padded z column p -> W2 row (or -1 for a zero-padding column)
__device__ __forceinline__ int w2_row(int p, int d, int NT) {
  const int e = 16 * NT;
  if (p < e) return p < d ? p : -1;
  return d + (p - e);  // me(8) ce(8) h(16) follow the item embedding
}

// LDS index of the B fragment quad (kb, col c, quad q). Quad q of column c
// sits at slot q ^ ((c >> 2) & 2) of the column's 64 B: each ds_read_b128
// lane group ({0-3,12-15,20-27}, {4-11,16-19,28-31}, and +32) then covers
// 16 distinct 16-B slots of the 256-B bank row (MI355X_MICROARCH.md §LDS).
__device__ __forceinline__ int wq_index(int kb, int c, int q, int dp) {
  return ((kb * dp + c) * 16) + 4 * (q ^ ((c >> 2) & 2));
}

// NTI: 16-column blocks of the (padded) item embedding in z; NT: output
// tiles of this pass, columns [col0, col0 + 16·NT). kLN: the pass covers
// every output column and applies the LayerNorm epilogue; otherwise it
// writes the pre-LN Dense output (z @ W2 + b2) of its columns (d = 256: two
// passes, then tt_ln_rows_kernel).
template <int NTI, int NT, bool kLN, bool kSave, int kFwdWaves>
__global__ __launch_bounds__(64 * kFwdWaves) void tt_item_forward_mfma_kernel(
    TTFwd P, const int32_t* __restrict__ item, const int32_t* __restrict__ man, const int32_t* __restrict__ cat,
    const float* __restrict__ numeric, int64_t n, int col0, float* __restrict__ out, float* __restrict__ z_save,
    float* __restrict__ xhat_save, float* __restrict__ rstd_save) {
  constexpr int dp = 16 * NT;
  constexpr int KB = NTI + 2;
  constexpr int kTG = NT >= 2 ? 2 : 1;
  constexpr bool kLds = true;
  extern __shared__ __attribute__((aligned(16))) float Ws[];  // [KB][dp][16]
  const int d = P.d, dz = P.d + 32;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = lane >> 4, m = lane & 15;
  // b2 | gamma | beta (zero-padded to dp) after the W2 fragments
  float* Vs = Ws + (kLds ? KB * dp * 16 : 0);
  if constexpr (kLds) {
    for (int o = threadIdx.x; o < KB * dp * 16; o += blockDim.x) {
      const int kb = o / (dp * 16), r = o % (dp * 16);
      const int c = r >> 4, qq = (r >> 2) & 3, j = r & 3;
      const int wr = w2_row(16 * kb + 4 * qq + j, d, NTI);
      Ws[wq_index(kb, c, qq, dp) + j] = (wr >= 0 && col0 + c < d) ? P.w2[(int64_t)wr * d + col0 + c] : 0.f;
    }
  }
  for (int o = threadIdx.x; o < 3 * dp; o += blockDim.x) {
    const int v = o / dp, c = o % dp;
    const float* src = v == 0 ? P.b2 : (v == 1 ? P.g : P.be);
    Vs[o] = col0 + c < d ? src[col0 + c] : 0.f;
  }
  __syncthreads();
  const bool vec = (d & 3) == 0;
  const int64_t tiles = (n + 15) >> 4;
  const int64_t stride = (int64_t)gridDim.x * kFwdWaves;
  // Per-lane row inputs of a tile (lane m's item), loaded one tile ahead;
  // the next tile's first two z blocks are gathered before this tile's
  // epilogue stores (on gfx950 vmcnt counts stores too: loads issued after
  // the stores would wait for them to drain).
  struct Row {
    int64_t ib;
    int mc;  // manufacturer (q < 2) or category row offset of this lane's quad
    float x0, x1;
  };
  auto load_row = [&](int64_t t) -> Row {
    int64_t r = t * 16 + m;
    r = r < n ? r : n - 1;
    Row o;
    o.ib = (int64_t)item[r] * d;
    o.mc = q < 2 ? man[r] * 8 + 4 * q : cat[r] * 8 + 4 * (q - 2);
    o.x0 = numeric[r * 2];
    o.x1 = numeric[r * 2 + 1];
    return o;
  };
  // block kb of an item's padded z (kb < NT: the item embedding, NT:
  // E_man | E_cat, NT + 1: h = relu(numeric @ W1 + b1)), this lane's quad
  auto block = [&](const Row& R, int kb) -> f4m {
    f4m v = f4m{0.f, 0.f, 0.f, 0.f};
    if constexpr (HREC_TT_FWD_ABLATE >= 2) return f4m{R.x0, R.x1, (float)kb, 1.f};
    if (kb < NTI) {
      const int c0 = 16 * kb + 4 * q;
      if (vec) {
        if (c0 < d) v = *reinterpret_cast<const f4m*>(P.ie + R.ib + c0);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = c0 + j < d ? P.ie[R.ib + c0 + j] : 0.f;
      }
    } else if (kb == NTI) {
      v = *reinterpret_cast<const f4m*>((q < 2 ? P.me : P.ce) + R.mc);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int hj = 4 * q + j;
        const float h = R.x0 * P.w1[hj] + R.x1 * P.w1[16 + hj] + P.b1[hj];
        v[j] = h > 0.f ? h : 0.f;
      }
    }
    return v;
  };
  int64_t tile = (int64_t)blockIdx.x * kFwdWaves + w;
  if (tile >= tiles) return;
  auto clampt = [&](int64_t t) { return t < tiles ? t : tile; };
  Row cur = load_row(tile), nxt = load_row(clampt(tile + stride));
  f4m a[KB];
  a[0] = block(cur, 0);
  a[1] = block(cur, 1);
  for (; tile < tiles; tile += stride) {
    const int64_t row = tile * 16 + m;  // lane m's item
    const bool live = row < n;
    // ---- Dense(d), transposed: C[out col][item] = W2^T z^T, so the C
    // layout gives lane (q, m) item m's output columns 16t + 4q + i. Fully
    // unrolled over the K blocks (the z blocks land in their own registers:
    // no moves, no vmcnt(0) drain per block); a scheduling barrier per block
    // keeps the compiler from hoisting every block's LDS reads at once.
    f4m acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f4m{0.f, 0.f, 0.f, 0.f};
    static_for<0, KB>([&](auto kbc) {
      constexpr int kb = decltype(kbc)::value;
      if constexpr (kb + 2 < KB) a[kb + 2] = block(cur, kb + 2);
      if constexpr (kSave) {
        if (live && col0 == 0) {  // z row in the backward pass's natural layout
          float* zr = z_save + row * dz;
          const int c0 = kb < NTI ? 16 * kb + 4 * q : (kb == NTI ? d + 4 * q : d + 16 + 4 * q);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (kb >= NTI || c0 + j < d) zr[c0 + j] = a[kb][j];
        }
      }
      // tiles in pairs, k-step outer inside a pair: consecutive MFMAs
      // alternate accumulators (the dependent-accumulator latency, 40 cycles,
      // exceeds the 32-cycle issue) while only two W2 fragments are live
#pragma unroll
      for (int t0 = 0; t0 < NT; t0 += kTG) {
        f4m b[kTG];
#pragma unroll
        for (int u = 0; u < kTG; ++u) {
          const int c = 16 * (t0 + u) + m;
          b[u] = *reinterpret_cast<const f4m*>(Ws + wq_index(kb, c, q, dp));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int u = 0; u < kTG; ++u)
            acc[t0 + u] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[u][j], a[kb][j], acc[t0 + u], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    const f4m p0 = block(nxt, 0), p1 = block(nxt, 1);
    const Row nn = load_row(clampt(tile + 2 * stride));
    if constexpr (HREC_TT_FWD_ABLATE >= 1) {
      float x = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) x += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
      if (x == 1234.5f) out[row] = x;
    } else if constexpr (!kLN) {
      if (live) {  // pre-LN Dense output of this pass's columns
        static_for<0, NT>([&](auto tc) {
          constexpr int t = decltype(tc)::value;
          const int c0 = 16 * t + 4 * q;
          const f4m bb = *reinterpret_cast<const f4m*>(Vs + c0);
          if (col0 + c0 < d) *reinterpret_cast<f4m*>(out + row * d + col0 + c0) = acc[t] + bb;
        });
      }
    } else {
      // ---- epilogue: + b2, LayerNormalization over item m's d columns
      // (in-lane over t, i; then across its 4 lanes q), y = xhat·gamma + beta
      float s = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int c0 = 16 * t + 4 * q;
        const f4m bb = *reinterpret_cast<const f4m*>(Vs + c0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[t][i] += bb[i];
          if (c0 + i < d) s += acc[t][i];
        }
      }
      s += __shfl_xor(s, 16, kWave);
      s += __shfl_xor(s, 32, kWave);
      const float mean = s / (float)d;
      float qv = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float x = acc[t][i] - mean;
          if (16 * t + 4 * q + i < d) qv += x * x;
        }
      }
      qv += __shfl_xor(qv, 16, kWave);
      qv += __shfl_xor(qv, 32, kWave);
      const float rstd = 1.0f / sqrtf(qv / (float)d + kLnEpsM);
      if (live) {
        float* orow = out + row * d;
        static_for<0, NT>([&](auto tc) {
          constexpr int t = decltype(tc)::value;
          const int c0 = 16 * t + 4 * q;
          const f4m gm = *reinterpret_cast<const f4m*>(Vs + dp + c0);
          const f4m bt = *reinterpret_cast<const f4m*>(Vs + 2 * dp + c0);
          f4m y, xh;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            xh[i] = (acc[t][i] - mean) * rstd;
            y[i] = xh[i] * gm[i] + bt[i];
          }
          if (vec) {
            if (c0 < d) {
              *reinterpret_cast<f4m*>(orow + c0) = y;
              if constexpr (kSave) *reinterpret_cast<f4m*>(xhat_save + row * d + c0) = xh;
            }
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              if (c0 + i >= d) continue;
              orow[c0 + i] = y[i];
              if constexpr (kSave) xhat_save[row * d + c0 + i] = xh[i];
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        });
        if constexpr (kSave) {
          if (q == 0) rstd_save[row] = rstd;
        }
      }
    }
    cur = nxt;
    nxt = nn;
    a[0] = p0;
    a[1] = p1;
  }
}

static int nt_of(int d) {
  if (d <= 16) return 1;
  if (d <= 32) return 2;
  if (d <= 64) return 4;
  if (d <= 128) return 8;
  if (d <= 256) return 16;
  return 0;
}

template <int NTI, int NT, bool kLN, bool kSave>
static int launch_fwd(const TTFwd& P, const int32_t* item, const int32_t* man, const int32_t* cat,
                      const float* numeric, int64_t n, int col0, float* out, float* z, float* xh, float* rs,
                      hipStream_t s) {
  // W2 (the pass's columns) + b2/gamma/beta in LDS, one persistent
  // 1024-thread workgroup per CU (81.5 KB at d = 128, 149 KB per d = 256 pass)
  constexpr int kW = 16;
  const size_t sm = ((size_t)(NTI + 2) * 16 * NT * 16 + 3 * 16 * NT) * sizeof(float);
  const int64_t tiles = (n + 15) / 16;
  int64_t grid = (tiles + kW - 1) / kW;
  if (grid > 256) grid = 256;
  hipLaunchKernelGGL((tt_item_forward_mfma_kernel<NTI, NT, kLN, kSave, kW>), dim3((unsigned)grid), dim3(64 * kW),
                     sm, s, P, item, man, cat, numeric, n, col0, out, z, xh, rs);
  return check_launch("tt_item_forward_mfma_kernel");
}

// LayerNorm of pre-LN rows in place (d = 256 path), one wave per row; same
// two-pass arithmetic as the fused epilogue.
__global__ __launch_bounds__(256) void tt_ln_rows_kernel(float* __restrict__ x, int64_t n, int d,
                                                         const float* __restrict__ g, const float* __restrict__ be,
                                                         float* __restrict__ xhat_save, float* __restrict__ rstd_save) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  float* xr = x + r * d;
  float s = 0.f;
  for (int c = lane; c < d; c += kWave) s += xr[c];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, kWave);
  const float mean = s / (float)d;
  float qv = 0.f;
  for (int c = lane; c < d; c += kWave) {
    const float t = xr[c] - mean;
    qv += t * t;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) qv += __shfl_xor(qv, off, kWave);
  const float rstd = 1.0f / sqrtf(qv / (float)d + kLnEpsM);
  for (int c = lane; c < d; c += kWave) {
    const float xh = (xr[c] - mean) * rstd;
    xr[c] = xh * g[c] + be[c];
    if (xhat_save) xhat_save[r * d + c] = xh;
  }
  if (rstd_save && lane == 0) rstd_save[r] = rstd;
}

}  // namespace hrec

// Called by hrec_tt_item_forward / hrec_tt_forward_backward (csrc/tt.hip)
// for d <= 256; returns 1 when d needs the scalar kernel instead.
int hrec_tt_item_forward_mfma(int d, const float* ie, const float* me, const float* ce, const float* w1,
                              const float* b1, const float* w2, const float* b2, const float* gamma,
                              const float* beta, const int32_t* item, const int32_t* man, const int32_t* cat,
                              const float* numeric, int64_t n, float* out, float* z_save, float* xhat_save,
                              float* rstd_save, void* stream) {
  using namespace hrec;
  const int NT = nt_of(d);
  if (NT == 0) return 1;
  TTFwd P{d, ie, me, ce, w1, b1, w2, b2, gamma, beta};
  hipStream_t s = as_stream(stream);
  const bool save = z_save != nullptr;
#define HREC_FWD_CASE(N)                                                                                 \
  case N:                                                                                                \
    return save ? launch_fwd<N, N, true, true>(P, item, man, cat, numeric, n, 0, out, z_save, xhat_save,  \
                                               rstd_save, s)                                             \
                : launch_fwd<N, N, true, false>(P, item, man, cat, numeric, n, 0, out, nullptr, nullptr,  \
                                                nullptr, s);
  switch (NT) {
    HREC_FWD_CASE(1)
    HREC_FWD_CASE(2)
    HREC_FWD_CASE(4)
    HREC_FWD_CASE(8)
    case 16: {  // two column passes (pre-LN) + LayerNorm rows
      int rc = save ? launch_fwd<16, 8, false, true>(P, item, man, cat, numeric, n, 0, out, z_save, nullptr,
                                                     nullptr, s)
                    : launch_fwd<16, 8, false, false>(P, item, man, cat, numeric, n, 0, out, nullptr, nullptr,
                                                      nullptr, s);
      if (rc) return rc;
      rc = launch_fwd<16, 8, false, false>(P, item, man, cat, numeric, n, 128, out, nullptr, nullptr, nullptr, s);
      if (rc) return rc;
      hipLaunchKernelGGL(tt_ln_rows_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, out, n, d, gamma, beta,
                         xhat_save, rstd_save);
      return check_launch("tt_ln_rows_kernel");
    }
  }
#undef HREC_FWD_CASE
  return 1;
}
