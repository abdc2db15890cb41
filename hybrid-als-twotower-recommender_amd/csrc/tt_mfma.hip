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
template <int NTI, int NT, bool kLN, bool kSave, int kFwdWaves, bool kLds>
__global__ __launch_bounds__(64 * kFwdWaves) void tt_item_forward_mfma_kernel(
    TTFwd P, const int32_t* __restrict__ item, const int32_t* __restrict__ man, const int32_t* __restrict__ cat,
    const float* __restrict__ numeric, int64_t n, int col0, float* __restrict__ out, float* __restrict__ z_save,
    float* __restrict__ xhat_save, float* __restrict__ rstd_save) {
  constexpr int dp = 16 * NT;
  constexpr int KB = NTI + 2;
  constexpr int kTG = NT >= 2 ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) float Ws[];  // [KB][dp][16] (kLds)
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
          if constexpr (kLds) {
            b[u] = *reinterpret_cast<const f4m*>(Ws + wq_index(kb, c, q, dp));
          } else {  // small calls: straight from W2 (L2-resident), no staging
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int wr = w2_row(16 * kb + 4 * q + j, d, NTI);
              b[u][j] = (wr >= 0 && col0 + c < d) ? P.w2[(int64_t)wr * d + col0 + c] : 0.f;
            }
          }
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

template <int NTI, int NT, bool kLN, bool kSave, int kW, bool kLds>
static int launch_fwd_w(const TTFwd& P, const int32_t* item, const int32_t* man, const int32_t* cat,
                        const float* numeric, int64_t n, int col0, float* out, float* z, float* xh, float* rs,
                        hipStream_t s) {
  const size_t sm = ((kLds ? (size_t)(NTI + 2) * 16 * NT * 16 : 0) + 3 * 16 * NT) * sizeof(float);
  const int64_t tiles = (n + 15) / 16;
  int64_t grid = (tiles + kW - 1) / kW;
  const int64_t cap = kW == 16 ? 256 : 4096;
  if (grid > cap) grid = cap;
  hipLaunchKernelGGL((tt_item_forward_mfma_kernel<NTI, NT, kLN, kSave, kW, kLds>), dim3((unsigned)grid), dim3(64 * kW),
                     sm, s, P, item, man, cat, numeric, n, col0, out, z, xh, rs);
  return check_launch("tt_item_forward_mfma_kernel");
}

// W2 (the pass's columns) + b2/gamma/beta in LDS. Catalogue-sized calls: one
// persistent 1024-thread workgroup per CU (81.5 KB at d = 128, 149 KB per
// d = 256 pass); small calls (a training batch): one wave per workgroup
// reading W2 straight from L2 (no staging), so the tiles spread over many
// CUs instead of queueing on one.
template <int NTI, int NT, bool kLN, bool kSave>
static int launch_fwd(const TTFwd& P, const int32_t* item, const int32_t* man, const int32_t* cat,
                      const float* numeric, int64_t n, int col0, float* out, float* z, float* xh, float* rs,
                      hipStream_t s) {
  if ((n + 15) / 16 >= 4096)
    return launch_fwd_w<NTI, NT, kLN, kSave, 16, true>(P, item, man, cat, numeric, n, col0, out, z, xh, rs, s);
  return launch_fwd_w<NTI, NT, kLN, kSave, 1, false>(P, item, man, cat, numeric, n, col0, out, z, xh, rs, s);
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

// ------------------------------------------------------------------------
// K6m: the backward pass of one Keras train step (MSE loss, batch B) with
// its two Dense(d) GEMMs on the f32 matrix cores. Three launches:
//   rows : per sample (one wave): score, dL/dscore = 2 (yhat - y) / B, the
//          LayerNorm backward of both towers -> dp [B, d] (grad of the item
//          Dense output) and the user-embedding row grads; squared / abs
//          error per sample;
//   dz   : dz = dp · W2^T [B, d+32] -> item / manufacturer / category row
//          grads and relu'(h) · dh = dpre [B, 16]   (MFMA, K = d);
//   dense: dW2 = z^T · dp [d+32, d]                    (MFMA, K = B) and
//          the column sums (db2, LN gamma/beta of both towers, dW1, db1,
//          loss sums) straight into the gradient block — no per-block
//          partials, one fixed summation order (deterministic).
// The k order inside the MFMA GEMMs is permuted as in K4m (16-B operand
// loads feed 4 k-steps).

namespace hrec {

struct TTBwd {
  int d;
  const float *w2, *gu, *gi;
};

// one wave per sample row
__global__ __launch_bounds__(256) void tt_bwd_rows_kernel(TTBwd P, const float* __restrict__ y, int64_t B,
                                                          const float* __restrict__ uvec,
                                                          const float* __restrict__ uxhat,
                                                          const float* __restrict__ urstd,
                                                          const float* __restrict__ ivec,
                                                          const float* __restrict__ ixhat,
                                                          const float* __restrict__ irstd, float* __restrict__ dp,
                                                          float* __restrict__ g_user, float* __restrict__ dyh,
                                                          float* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= B) return;
  const int d = P.d;
  const float* u = uvec + g * d;
  const float* v = ivec + g * d;
  float s = 0.f;
  for (int c = lane; c < d; c += kWave) s = fmaf(u[c], v[c], s);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, kWave);
  const float e = s - y[g];
  const float dy = 2.0f * e / (float)B;
  // item LN backward: dxh = dy·u·gamma ; dx = rstd·(dxh - mean(dxh) - xh·mean(dxh·xh))
  float m1 = 0.f, m2 = 0.f, u1 = 0.f, u2 = 0.f;
  for (int c = lane; c < d; c += kWave) {
    const float di = dy * u[c] * P.gi[c];
    m1 += di;
    m2 += di * ixhat[g * d + c];
    const float du = dy * v[c] * P.gu[c];
    u1 += du;
    u2 += du * uxhat[g * d + c];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    m1 += __shfl_xor(m1, off, kWave);
    m2 += __shfl_xor(m2, off, kWave);
    u1 += __shfl_xor(u1, off, kWave);
    u2 += __shfl_xor(u2, off, kWave);
  }
  m1 /= (float)d;
  m2 /= (float)d;
  u1 /= (float)d;
  u2 /= (float)d;
  const float ir = irstd[g], ur = urstd[g];
  for (int c = lane; c < d; c += kWave) {
    const float di = dy * u[c] * P.gi[c];
    dp[g * d + c] = ir * (di - m1 - ixhat[g * d + c] * m2);
    const float du = dy * v[c] * P.gu[c];
    g_user[g * d + c] = ur * (du - u1 - uxhat[g * d + c] * u2);
  }
  if (lane == 0) {
    dyh[g] = dy;
    err[2 * g] = e * e;
    err[2 * g + 1] = fabsf(e);
  }
}

// dz = dp · W2^T, transposed on the matrix cores: C[z col][sample] =
// W2 · dp^T, so lane (q, m) holds z columns 16t + 4q + i of sample 16·tile
// + m. One wave per 16 samples x all z columns (dz <= 288: NTZ <= 18).
template <int NTZ>
__global__ __launch_bounds__(64) void tt_bwd_dz_kernel(TTBwd P, int64_t B, const float* __restrict__ dp,
                                                       const float* __restrict__ zsave, float* __restrict__ g_item,
                                                       float* __restrict__ g_man, float* __restrict__ g_cat,
                                                       float* __restrict__ dpre) {
  const int d = P.d, dz = d + 32;
  const int lane = threadIdx.x, q = lane >> 4, m = lane & 15;
  const int64_t row = (int64_t)blockIdx.x * 16 + m;
  const bool live = row < B;
  const int64_t rr = live ? row : B - 1;
  f4m acc[NTZ];
#pragma unroll
  for (int t = 0; t < NTZ; ++t) acc[t] = f4m{0.f, 0.f, 0.f, 0.f};
  const int nkb = (d + 15) / 16;
  for (int kb = 0; kb < nkb; ++kb) {
    const int k0 = 16 * kb + 4 * q;
    f4m a;
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = k0 + j < d ? dp[rr * d + k0 + j] : 0.f;
#pragma unroll
    for (int t = 0; t < NTZ; ++t) {
      const int zc = 16 * t + m;  // A row = z column
      f4m b;
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = (zc < dz && k0 + j < d) ? P.w2[(int64_t)zc * d + k0 + j] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j], a[j], acc[t], 0, 0, 0);
    }
  }
  if (!live) return;
#pragma unroll
  for (int t = 0; t < NTZ; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 16 * t + 4 * q + i;
      const float x = acc[t][i];
      if (c < d) {
        g_item[row * d + c] = x;
      } else if (c < d + 8) {
        g_man[row * 8 + (c - d)] = x;
      } else if (c < d + 16) {
        g_cat[row * 8 + (c - d - 8)] = x;
      } else if (c < dz) {
        const float h = zsave[row * dz + c];
        dpre[row * 16 + (c - d - 16)] = h > 0.f ? x : 0.f;  // relu'
      }
    }
  }
}

// dW2 = z^T · dp over the batch, then the column sums. 1024-thread blocks:
// blocks [0, tiles) each own one 16 x 16 tile of dW2, its 16 waves split the
// batch (MFMA, K = the wave's samples in order 16kb + 4q + j) and the 16
// partial tiles are summed in LDS in wave order; the remaining blocks take
// 64 columns each of [db2 | dgi | dbi | dgu | dbu | dW1 | db1 | loss sums],
// 16 sample stripes per column summed the same way. Fixed orders throughout
// (deterministic), no per-block partials in HBM. Grad layout =
// tt_engine.dense_layout: W2[(d+32)·d] | b2 | gamma_i | beta_i | gamma_u |
// beta_u | W1[32] | b1[16] | sum sq err | sum abs err.
constexpr int kBwdWaves = 16;
__global__ __launch_bounds__(64 * kBwdWaves) void tt_bwd_dense_kernel(
    TTBwd P, int64_t B, const float* __restrict__ zsave, const float* __restrict__ dp,
    const float* __restrict__ uvec, const float* __restrict__ uxhat, const float* __restrict__ ivec,
    const float* __restrict__ ixhat, const float* __restrict__ dyh, const float* __restrict__ numeric,
    const float* __restrict__ dpre, const float* __restrict__ err, float* __restrict__ grad) {
  __shared__ float red[kBwdWaves][256];
  const int d = P.d, dz = d + 32;
  const int tz = (dz + 15) / 16, td = (d + 15) / 16;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int blk = blockIdx.x;
  if (blk < tz * td) {
    const int q = lane >> 4, m = lane & 15;
    const int zt = blk / td, dt = blk % td;
    const int zc = 16 * zt + m, dc = 16 * dt + m;
    const int64_t per = ((B + kBwdWaves - 1) / kBwdWaves + 15) / 16 * 16;  // samples per wave
    const int64_t sb = w * per, se = sb + per < B ? sb + per : B;
    f4m acc = f4m{0.f, 0.f, 0.f, 0.f};
    for (int64_t s0 = sb; s0 < se; s0 += 16) {
      f4m a, b;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t s = s0 + 4 * q + j;
        a[j] = (s < se && zc < dz) ? zsave[s * dz + zc] : 0.f;
        b[j] = (s < se && dc < d) ? dp[s * d + dc] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) red[w][(4 * q + i) * 16 + m] = acc[i];  // C[z 4q + i][d m]
    __syncthreads();
    if (threadIdx.x < 256) {
      const int zr = 16 * zt + (threadIdx.x >> 4), c = 16 * dt + (threadIdx.x & 15);
      float sum = 0.f;
#pragma unroll
      for (int v = 0; v < kBwdWaves; ++v) sum += red[v][threadIdx.x];
      if (zr < dz && c < d) grad[(int64_t)zr * d + c] = sum;
    }
    return;
  }
  float* tail = grad + (int64_t)dz * d;
  const int ncol = 5 * d + 48 + 2;
  const int o = (blk - tz * td) * 64 + lane;  // column of this lane; w = sample stripe
  float acc = 0.f;
  if (o < 5 * d) {
    const int kind = o / d, j = o % d;
    for (int64_t s = w; s < B; s += kBwdWaves) {
      const float dy = dyh[s];
      if (kind == 0) {
        acc += dp[s * d + j];
      } else if (kind == 1 || kind == 2) {
        const float dvi = dy * uvec[s * d + j];  // d item_vec
        acc = kind == 1 ? fmaf(dvi, ixhat[s * d + j], acc) : acc + dvi;
      } else {
        const float dvu = dy * ivec[s * d + j];  // d user_vec
        acc = kind == 3 ? fmaf(dvu, uxhat[s * d + j], acc) : acc + dvu;
      }
    }
  } else if (o < 5 * d + 32) {  // dW1[i][j] = sum_s x_i · dpre_j
    const int i = (o - 5 * d) / 16, j = (o - 5 * d) % 16;
    for (int64_t s = w; s < B; s += kBwdWaves) acc = fmaf(numeric[s * 2 + i], dpre[s * 16 + j], acc);
  } else if (o < 5 * d + 48) {
    const int j = o - 5 * d - 32;
    for (int64_t s = w; s < B; s += kBwdWaves) acc += dpre[s * 16 + j];
  } else if (o < ncol) {
    const int k = o - 5 * d - 48;
    for (int64_t s = w; s < B; s += kBwdWaves) acc += err[2 * s + k];
  }
  red[w][lane] = acc;
  __syncthreads();
  if (threadIdx.x < 64 && o < ncol) {
    float sum = 0.f;
#pragma unroll
    for (int v = 0; v < kBwdWaves; ++v) sum += red[v][threadIdx.x];
    tail[o] = sum;
  }
}

}  // namespace hrec

// Called by hrec_tt_forward_backward (csrc/tt.hip) after both forwards:
// returns 1 when d needs the scalar backward instead (d > 256).
int hrec_tt_backward_mfma(int d, const float* w2, const float* gamma_u, const float* gamma_i, const float* y,
                          int64_t B, const float* uvec, const float* uxhat, const float* urstd, const float* ivec,
                          const float* ixhat, const float* irstd, const float* zsave, const float* numeric,
                          float* g_user, float* g_item, float* g_man, float* g_cat, float* grad, float* scratch,
                          void* stream) {
  using namespace hrec;
  if (d > 256) return 1;
  hipStream_t s = as_stream(stream);
  TTBwd P{d, w2, gamma_u, gamma_i};
  float* dp = scratch;               // [B, d]
  float* dpre = dp + B * d;          // [B, 16]
  float* dyh = dpre + B * 16;        // [B]
  float* err = dyh + B;              // [B, 2]
  hipLaunchKernelGGL(tt_bwd_rows_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, P, y, B, uvec, uxhat, urstd,
                     ivec, ixhat, irstd, dp, g_user, dyh, err);
  int rc = check_launch("tt_bwd_rows_kernel");
  if (rc) return rc;
  const int ntz = (d + 32 + 15) / 16;
  const dim3 gz((unsigned)((B + 15) / 16));
#define HREC_DZ_CASE(N)                                                                                          \
  case N:                                                                                                        \
    hipLaunchKernelGGL(tt_bwd_dz_kernel<N>, gz, dim3(64), 0, s, P, B, dp, zsave, g_item, g_man, g_cat, dpre); \
    break;
  switch (ntz) {
    HREC_DZ_CASE(3) HREC_DZ_CASE(4) HREC_DZ_CASE(5) HREC_DZ_CASE(6) HREC_DZ_CASE(7) HREC_DZ_CASE(8)
    HREC_DZ_CASE(9) HREC_DZ_CASE(10) HREC_DZ_CASE(11) HREC_DZ_CASE(12) HREC_DZ_CASE(13) HREC_DZ_CASE(14)
    HREC_DZ_CASE(15) HREC_DZ_CASE(16) HREC_DZ_CASE(17) HREC_DZ_CASE(18)
    default:
      return 1;
  }
#undef HREC_DZ_CASE
  rc = check_launch("tt_bwd_dz_kernel");
  if (rc) return rc;
  const int tiles = ntz * ((d + 15) / 16);
  const int sums = (5 * d + 48 + 2 + 63) / 64;
  hipLaunchKernelGGL(tt_bwd_dense_kernel, dim3((unsigned)(tiles + sums)), dim3(64 * kBwdWaves), 0, s, P, B, zsave, dp, uvec,
                     uxhat, ivec, ixhat, dyh, numeric, dpre, err, grad);
  return check_launch("tt_bwd_dense_kernel");
}
