// K4-K7: the two-tower model of src/two_tower_model.py:38-89 on gfx950.
//
//   user_vec = LN_u(E_user[u])                                   (:71-74)
//   h        = relu(numeric @ W1 + b1)        Dense(16, relu)    (:56-57)
//   z        = [E_item[i] | E_man[m] | E_cat[c] | h]  (d+32)      (:60)
//   item_vec = LN_i(z @ W2 + b2)              Dense(d) + LN      (:63-64)
//   score    = <user_vec, item_vec>           Dot(axes=1)        (:80)
// LayerNormalization: Keras 2.8 (epsilon 1e-3, biased variance over the
// last axis, y = xhat*gamma + beta). Loss MSE, optimiser Adam (:84-88) with
// TF 2.8's dense ResourceApplyAdam and sparse (IndexedSlices) update rules.
// f32 throughout (the reference's Keras dtype).
#include "common.h"

namespace hrec {

constexpr int kTR = 8;      // rows (samples / candidates) per workgroup: 32 workgroups at a batch of 256
constexpr int kBlock = 256;
constexpr float kLnEps = 1e-3f;

struct TTDev {
  int d;
  const float *ue, *ie, *me, *ce, *w1, *b1, *w2, *b2, *gu, *bu, *gi, *bi;
};

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, kWave);
  return x;
}

// LayerNorm of one row held in LDS (length d), one wave. Writes y (and the
// normalised row + 1/std when save != nullptr).
__device__ __forceinline__ void ln_row(const float* __restrict__ x, int d, const float* __restrict__ gamma,
                                       const float* __restrict__ beta, float* __restrict__ y,
                                       float* __restrict__ xhat_out, float* __restrict__ rstd_out, int lane) {
  float s = 0.f;
  for (int c = lane; c < d; c += kWave) s += x[c];
  const float mean = wave_sum(s) / (float)d;
  float q = 0.f;
  for (int c = lane; c < d; c += kWave) {
    const float t = x[c] - mean;
    q += t * t;
  }
  const float var = wave_sum(q) / (float)d;
  const float rstd = 1.0f / sqrtf(var + kLnEps);
  for (int c = lane; c < d; c += kWave) {
    const float xh = (x[c] - mean) * rstd;
    y[c] = xh * gamma[c] + beta[c];
    if (xhat_out) xhat_out[c] = xh;
  }
  if (rstd_out && lane == 0) *rstd_out = rstd;
}

// K4: item tower for n rows. Optional saves for the backward pass:
// z [n, d+32], xhat [n, d], rstd [n].
__global__ __launch_bounds__(kBlock) void tt_item_forward_kernel(TTDev P, const int32_t* __restrict__ item,
                                                                  const int32_t* __restrict__ man,
                                                                  const int32_t* __restrict__ cat,
                                                                  const float* __restrict__ numeric, int64_t n,
                                                                  float* __restrict__ out, float* __restrict__ z_save,
                                                                  float* __restrict__ xhat_save,
                                                                  float* __restrict__ rstd_save) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int d = P.d, dz = P.d + 32;
  float* zs = smem;              // [kTR][dz]
  float* ps = smem + kTR * dz;   // [kTR][d]
  const int64_t r0 = (int64_t)blockIdx.x * kTR;
  const int rows = (int)((n - r0) < kTR ? (n - r0) : kTR);
  // gather the concat input
  for (int o = threadIdx.x; o < kTR * dz; o += blockDim.x) {
    const int r = o / dz, c = o % dz;
    float v = 0.f;
    if (r < rows) {
      const int64_t g = r0 + r;
      if (c < d) {
        v = P.ie[(int64_t)item[g] * d + c];
      } else if (c < d + 8) {
        v = P.me[(int64_t)man[g] * 8 + (c - d)];
      } else if (c < d + 16) {
        v = P.ce[(int64_t)cat[g] * 8 + (c - d - 8)];
      } else {
        const int j = c - d - 16;
        const float x0 = numeric[g * 2], x1 = numeric[g * 2 + 1];
        const float h = x0 * P.w1[j] + x1 * P.w1[16 + j] + P.b1[j];
        v = h > 0.f ? h : 0.f;
      }
    }
    zs[o] = v;
  }
  __syncthreads();
  // Dense(d): p = z @ W2 + b2 (W2 [dz][d] row-major, column reads coalesced)
  for (int o = threadIdx.x; o < kTR * d; o += blockDim.x) {
    const int r = o / d, j = o % d;
    const float* zr = zs + r * dz;
    float acc = 0.f;
    for (int k = 0; k < dz; ++k) acc = fmaf(zr[k], P.w2[(int64_t)k * d + j], acc);
    ps[o] = acc + P.b2[j];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int r = w; r < rows; r += kBlock / 64) {
    const int64_t g = r0 + r;
    ln_row(ps + r * d, d, P.gi, P.bi, out + g * d, xhat_save ? xhat_save + g * d : nullptr,
           rstd_save ? rstd_save + g : nullptr, lane);
  }
  if (z_save) {
    for (int o = threadIdx.x; o < rows * dz; o += blockDim.x) z_save[r0 * dz + o] = zs[o];
  }
}

// K5: user tower.
__global__ __launch_bounds__(kBlock) void tt_user_forward_kernel(TTDev P, const int32_t* __restrict__ user,
                                                                  int64_t n, float* __restrict__ out,
                                                                  float* __restrict__ xhat_save,
                                                                  float* __restrict__ rstd_save) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (g >= n) return;
  const int d = P.d;
  ln_row(P.ue + (int64_t)user[g] * d, d, P.gu, P.bu, out + g * d, xhat_save ? xhat_save + g * d : nullptr,
         rstd_save ? rstd_save + g : nullptr, lane);
}

// The one f32 summation order of every two-tower score (Dot(axes=1)), so a
// score's bits do not depend on the batch, the kernel or the call that
// produced it: an fmaf chain from zero (v_mfma_f32_16x16x4_f32 is that chain
// bit for bit, MI355X_MICROARCH.md) over k in
//   d in {32, 64, 128, 256}: hrec_dot_scores' order, steps of 16, inside a
//     step k = 16 ks + 4 g + e with g fastest (csrc/dot_topk.hip, dot_gemv.hip);
//   any other d: k = 0, 1, .., d - 1 (tt_score_mfma*_kernel: k = 4 ks + g).
__host__ __device__ inline bool tt_dot_order(int d) { return d == 32 || d == 64 || d == 128 || d == 256; }
__device__ __forceinline__ float tt_chain_dot(const float* __restrict__ u, const float* __restrict__ v, int d) {
  float acc = 0.f;
  if (tt_dot_order(d)) {
    for (int k0 = 0; k0 < d; k0 += 16)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc = fmaf(u[k0 + 4 * g + e], v[k0 + 4 * g + e], acc);
  } else {
    for (int c = 0; c < d; ++c) acc = fmaf(u[c], v[c], acc);
  }
  return acc;
}

// Dot(axes=1): out[b*N + j] = <U[b], V[j]>, one thread per (b, j)
// (few users, or operands the matrix-core kernels cannot load).
__global__ __launch_bounds__(kBlock) void tt_score_kernel(const float* __restrict__ U, int B,
                                                          const float* __restrict__ V, int64_t N, int d,
                                                          float* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (j >= N || b >= B) return;
  out[(int64_t)b * N + j] = tt_chain_dot(U + (int64_t)b * d, V + j * d, d);
}

// K8: all-pairs Dot(axes=1) on the matrix cores, out[b*N + j] = <U[b], V[j]>.
// v_mfma_f32_16x16x4_f32 (exact f32 fma chain per k-step), 64 users x 64
// items per 256-thread block, the d axis staged through LDS in chunks of 64
// (rows padded to 65 floats: conflict-free column reads).
typedef float f4v __attribute__((ext_vector_type(4)));
#ifndef HREC_TT_SCORE_STORE
#define HREC_TT_SCORE_STORE 0  // score tile stores: 0 plain, 1 non-temporal, 2 none (timing-only build)
#endif
#ifndef HREC_TT_SCORE_DIRECT
#define HREC_TT_SCORE_DIRECT 0  // 1 = scores stored from the MFMA C layout (measured slower: hybrid 0.31 -> 0.32 ms)
#endif
__global__ __launch_bounds__(256) void tt_score_mfma_kernel(const float* __restrict__ U, int B,
                                                            const float* __restrict__ V, int64_t N, int d,
                                                            float* __restrict__ out) {
  // One 64-item tile per block; the block walks every 64-user tile, so each
  // item vector is read from HBM once (the user vectors stay in L2).
  __shared__ float Us[64][65];
  __shared__ float Vs[64][65];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t j0 = (int64_t)blockIdx.x * 64;
  const bool vec = (N % 4 == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
  for (int b0 = 0; b0 < B; b0 += 64) {
    f4v acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f4v{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < d; k0 += 64) {
      __syncthreads();  // the previous tile's readers are done with Us/Vs
      for (int o = threadIdx.x; o < 64 * 64; o += 256) {
        const int r = o >> 6, c = o & 63;
        const int kk = k0 + c;
        Us[r][c] = (b0 + r < B && kk < d) ? U[(int64_t)(b0 + r) * d + kk] : 0.f;
        if (b0 == 0 || d > 64) Vs[r][c] = (j0 + r < N && kk < d) ? V[(j0 + r) * d + kk] : 0.f;
      }
      __syncthreads();
#pragma unroll 4
      for (int ks = 0; ks < 16; ++ks) {
        const float a = Us[16 * w + (lane & 15)][4 * ks + (lane >> 4)];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float b = Vs[16 * t + (lane & 15)][4 * ks + (lane >> 4)];
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
        }
      }
    }
    if constexpr (HREC_TT_SCORE_DIRECT) {
      // straight from the C layout: lane holds users 16w + 4(lane>>4) + r,
      // item 16t + (lane & 15) -> 64-B runs per user row, no LDS round trip
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int64_t j = j0 + 16 * t + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int b = b0 + 16 * w + 4 * (lane >> 4) + r;
          if (b < B && j < N) out[(int64_t)b * N + j] = acc[t][r];
        }
      }
      continue;
    }
    // stage the 64 x 64 tile in LDS (over Us), then write each user's 64
    // items as 256 contiguous bytes (16 lanes x float4)
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) Us[16 * w + 4 * (lane >> 4) + r][16 * t + (lane & 15)] = acc[t][r];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int o = q * 256 + threadIdx.x;
      const int row = o >> 4, c4 = (o & 15) * 4;
      const int b = b0 + row;
      const int64_t j = j0 + c4;
      if (b >= B) continue;
      float* dst = out + (int64_t)b * N + j;
      if (vec && j + 3 < N) {
        const float4 v4 = make_float4(Us[row][c4], Us[row][c4 + 1], Us[row][c4 + 2], Us[row][c4 + 3]);
        if constexpr (HREC_TT_SCORE_STORE == 0) {
          *reinterpret_cast<float4*>(dst) = v4;
        } else if constexpr (HREC_TT_SCORE_STORE == 1) {  // streaming (non-temporal) store
          __builtin_nontemporal_store(v4.x, dst);
          __builtin_nontemporal_store(v4.y, dst + 1);
          __builtin_nontemporal_store(v4.z, dst + 2);
          __builtin_nontemporal_store(v4.w, dst + 3);
        } else {  // timing-only: no store unless the value is impossible
          if (v4.x == 1234.5f && v4.y == -1234.5f) *reinterpret_cast<float4*>(dst) = v4;
        }
      } else {
        for (int e = 0; e < 4; ++e)
          if (j + e < N) dst[e] = Us[row][c4 + e];
      }
    }
  }
}

// The same products in the same k order (one exact f32 fma chain over k per
// score, so bit-identical), staged with 16-B loads (d % 4 == 0, 16-B aligned
// rows): 4 instead of 16 staging iterations per tile and array, and rows
// padded to 66 floats so the operand reads (row + 4 ks + g) hit 32 distinct
// banks per 32-lane half.
#ifndef HREC_TT_SCORE_V2
#define HREC_TT_SCORE_V2 1
#endif
constexpr int kTs2 = 66;
__global__ __launch_bounds__(256) void tt_score_mfma2_kernel(const float* __restrict__ U, int B,
                                                             const float* __restrict__ V, int64_t N, int d,
                                                             float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float Us[64 * kTs2];
  __shared__ __attribute__((aligned(16))) float Vs[64 * kTs2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t j0 = (int64_t)blockIdx.x * 64;
  const bool vec = (N % 4 == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
  auto stage = [&](float* dst, const float* __restrict__ src, int64_t row0, int64_t nrows, int k0) {
    for (int o = threadIdx.x; o < 64 * 16; o += 256) {
      const int r = o >> 4, c4 = (o & 15) * 4;
      const int kk = k0 + c4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row0 + r < nrows && kk < d) v = *reinterpret_cast<const float4*>(src + (row0 + r) * d + kk);
      float2* p = reinterpret_cast<float2*>(dst + r * kTs2 + c4);
      p[0] = make_float2(v.x, v.y);
      p[1] = make_float2(v.z, v.w);
    }
  };
  for (int b0 = 0; b0 < B; b0 += 64) {
    f4v acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f4v{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < d; k0 += 64) {
      __syncthreads();  // the previous tile's readers are done with Us/Vs
      stage(Us, U, b0, B, k0);
      if (b0 == 0 || d > 64) stage(Vs, V, j0, N, k0);
      __syncthreads();
#pragma unroll 4
      for (int ks = 0; ks < 16; ++ks) {
        const float a = Us[(16 * w + (lane & 15)) * kTs2 + 4 * ks + (lane >> 4)];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float b = Vs[(16 * t + (lane & 15)) * kTs2 + 4 * ks + (lane >> 4)];
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) Us[(16 * w + 4 * (lane >> 4) + r) * kTs2 + 16 * t + (lane & 15)] = acc[t][r];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int o = q * 256 + threadIdx.x;
      const int row = o >> 4, c4 = (o & 15) * 4;
      const int b = b0 + row;
      const int64_t j = j0 + c4;
      if (b >= B) continue;
      const float2* p = reinterpret_cast<const float2*>(Us + row * kTs2 + c4);
      const float2 x0 = p[0], x1 = p[1];
      float* dst = out + (int64_t)b * N + j;
      if (vec && j + 3 < N) {
        *reinterpret_cast<float4*>(dst) = make_float4(x0.x, x0.y, x1.x, x1.y);
      } else {
        const float xs[4] = {x0.x, x0.y, x1.x, x1.y};
        for (int e = 0; e < 4; ++e)
          if (j + e < N) dst[e] = xs[e];
      }
    }
  }
}

// Paired dot: out[r] = <U[r], V[r]> (model.predict on per-row inputs), in
// the ranking scores' order (tt_chain_dot): a pair predicted here has the
// bits the same pair gets in hrec_tt_score. One thread per row.
__global__ __launch_bounds__(kBlock) void tt_pair_score_kernel(const float* __restrict__ U,
                                                               const float* __restrict__ V, int64_t n, int d,
                                                               float* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= n) return;
  out[r] = tt_chain_dot(U + r * d, V + r * d, d);
}

// Backward of one training batch, kTR samples per workgroup. Inputs are the
// forward saves; outputs: per-sample embedding-row grads and per-block
// partial sums of the dense-parameter grads (reduced in fixed block order by
// tt_reduce_partials -> deterministic).
//
// partial layout per block (floats): dW2[dz*d] | db2[d] | dgi[d] | dbi[d] |
//                                    dgu[d] | dbu[d] | dW1[32] | db1[16] | sq_err[1] | abs_err[1]
__global__ __launch_bounds__(kBlock) void tt_backward_kernel(
    TTDev P, const float* __restrict__ y, int64_t B, const float* __restrict__ uvec,
    const float* __restrict__ uxhat, const float* __restrict__ urstd, const float* __restrict__ ivec,
    const float* __restrict__ ixhat, const float* __restrict__ irstd, const float* __restrict__ zsave,
    const float* __restrict__ numeric, float* __restrict__ g_user, float* __restrict__ g_item,
    float* __restrict__ g_man, float* __restrict__ g_cat, float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int d = P.d, dz = P.d + 32;
  const int64_t r0 = (int64_t)blockIdx.x * kTR;
  const int rows = (int)((B - r0) < kTR ? (B - r0) : kTR);
  float* dp = smem;                  // [kTR][d]  grad of the Dense(d) output
  float* dpre = dp + kTR * d;        // [kTR][16] grad of the Dense(16) pre-activation
  float* dyh = dpre + kTR * 16;      // [kTR]     dL/dscore
  float* red = dyh + kTR;            // [8]: sq err, abs err per wave
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const size_t plen = (size_t)dz * d + 5 * (size_t)d + 48 + 2;
  float* part = partial + (size_t)blockIdx.x * plen;

  // score, MSE grad, LN backward (item -> dp, user -> g_user)
  float loss_acc = 0.f, abs_acc = 0.f;
  for (int r = w; r < kTR; r += kBlock / 64) {
    if (r >= rows) {
      for (int c = lane; c < d; c += kWave) dp[r * d + c] = 0.f;
      if (lane == 0) dyh[r] = 0.f;
      continue;
    }
    const int64_t g = r0 + r;
    float s = 0.f;
    for (int c = lane; c < d; c += kWave) s = fmaf(uvec[g * d + c], ivec[g * d + c], s);
    const float yhat = wave_sum(s);
    const float e = yhat - y[g];
    const float dy = 2.0f * e / (float)B;
    if (lane == 0) {
      dyh[r] = dy;
      loss_acc += e * e;
      abs_acc += fabsf(e);
    }
    // item LN backward: dxh = dy*u*gamma ; dx = rstd*(dxh - mean(dxh) - xh*mean(dxh*xh))
    float m1 = 0.f, m2 = 0.f;
    for (int c = lane; c < d; c += kWave) {
      const float dxh = dy * uvec[g * d + c] * P.gi[c];
      m1 += dxh;
      m2 += dxh * ixhat[g * d + c];
    }
    m1 = wave_sum(m1) / (float)d;
    m2 = wave_sum(m2) / (float)d;
    for (int c = lane; c < d; c += kWave) {
      const float xh = ixhat[g * d + c];
      const float dxh = dy * uvec[g * d + c] * P.gi[c];
      dp[r * d + c] = irstd[g] * (dxh - m1 - xh * m2);
    }
    float u1 = 0.f, u2 = 0.f;
    for (int c = lane; c < d; c += kWave) {
      const float dxh = dy * ivec[g * d + c] * P.gu[c];
      u1 += dxh;
      u2 += dxh * uxhat[g * d + c];
    }
    u1 = wave_sum(u1) / (float)d;
    u2 = wave_sum(u2) / (float)d;
    for (int c = lane; c < d; c += kWave) {
      const float xh = uxhat[g * d + c];
      const float dxh = dy * ivec[g * d + c] * P.gu[c];
      g_user[g * d + c] = urstd[g] * (dxh - u1 - xh * u2);
    }
  }
  if (lane == 0) {
    red[w] = loss_acc;
    red[4 + w] = abs_acc;
  }
  __syncthreads();
  // dz = dp @ W2^T -> item / manufacturer / category rows, and dh -> dpre
  for (int o = threadIdx.x; o < kTR * dz; o += blockDim.x) {
    const int r = o / dz, k = o % dz;
    if (r >= rows) {
      if (k >= d + 16) dpre[r * 16 + (k - d - 16)] = 0.f;
      continue;
    }
    const int64_t g = r0 + r;
    const float* dpr = dp + r * d;
    const float* w2r = P.w2 + (int64_t)k * d;
    float acc = 0.f;
    for (int j = 0; j < d; ++j) acc = fmaf(dpr[j], w2r[j], acc);
    if (k < d) {
      g_item[g * d + k] = acc;
    } else if (k < d + 8) {
      g_man[g * 8 + (k - d)] = acc;
    } else if (k < d + 16) {
      g_cat[g * 8 + (k - d - 8)] = acc;
    } else {
      const int j = k - d - 16;
      const float h = zsave[g * dz + k];
      dpre[r * 16 + j] = h > 0.f ? acc : 0.f;  // relu'
    }
  }
  __syncthreads();
  // dense partials over this block's rows (fixed row order)
  for (int o = threadIdx.x; o < dz * d; o += blockDim.x) {
    const int k = o / d, j = o % d;
    float acc = 0.f;
    for (int r = 0; r < rows; ++r) acc = fmaf(zsave[(r0 + r) * dz + k], dp[r * d + j], acc);
    part[o] = acc;
  }
  for (int j = threadIdx.x; j < d; j += blockDim.x) {
    float db2 = 0.f, dgi = 0.f, dbi = 0.f, dgu = 0.f, dbu = 0.f;
    for (int r = 0; r < rows; ++r) {
      const int64_t g = r0 + r;
      const float dy = dyh[r];
      const float dvi = dy * uvec[g * d + j];  // d item_vec
      const float dvu = dy * ivec[g * d + j];  // d user_vec
      db2 += dp[r * d + j];
      dgi = fmaf(dvi, ixhat[g * d + j], dgi);
      dbi += dvi;
      dgu = fmaf(dvu, uxhat[g * d + j], dgu);
      dbu += dvu;
    }
    float* q = part + (size_t)dz * d;
    q[j] = db2;
    q[d + j] = dgi;
    q[2 * d + j] = dbi;
    q[3 * d + j] = dgu;
    q[4 * d + j] = dbu;
  }
  if (threadIdx.x < 48) {
    float* q = part + (size_t)dz * d + 5 * (size_t)d;
    float acc = 0.f;
    if (threadIdx.x < 32) {  // dW1[i][j] = sum_r x_i * dpre_j
      const int i = threadIdx.x / 16, j = threadIdx.x % 16;
      for (int r = 0; r < rows; ++r) acc = fmaf(numeric[(r0 + r) * 2 + i], dpre[r * 16 + j], acc);
    } else {
      const int j = threadIdx.x - 32;
      for (int r = 0; r < rows; ++r) acc += dpre[r * 16 + j];
    }
    q[threadIdx.x] = acc;
  }
  if (threadIdx.x == 0) {
    part[plen - 2] = red[0] + red[1] + red[2] + red[3];
    part[plen - 1] = red[4] + red[5] + red[6] + red[7];
  }
}

__global__ __launch_bounds__(kBlock) void tt_reduce_partials_kernel(const float* __restrict__ partial, int nblk,
                                                                     size_t plen, float* __restrict__ out) {
  const size_t o = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= plen) return;
  float acc = 0.f;
  for (int b = 0; b < nblk; ++b) acc += partial[(size_t)b * plen + o];
  out[o] = acc;
}

// ---------------------------------------------------------------- Adam
// TF ResourceApplyAdam (dense): m += (g-m)*(1-b1); v += (g^2-v)*(1-b2);
// var -= (m*alpha)/(sqrt(v)+eps), alpha = lr*sqrt(1-b2^t)/(1-b1^t) (host f32).
__global__ __launch_bounds__(kBlock) void adam_dense_kernel(float* __restrict__ var, float* __restrict__ m,
                                                             float* __restrict__ v, const float* __restrict__ g,
                                                             int64_t n, float alpha, float b1, float b2, float eps) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= n) return;
  const float gr = g[o];
  float mo = m[o], vo = v[o];
  mo += (gr - mo) * (1.0f - b1);
  vo += (gr * gr - vo) * (1.0f - b2);
  m[o] = mo;
  v[o] = vo;
  var[o] -= (mo * alpha) / (sqrtf(vo) + eps);
}

// IndexedSlices dedup (tf.unique order = first occurrence, segment sums in
// sample order): gsum row q is the summed grad of sample q when q is the
// first occurrence of its index; mark[idx] = q.
// One wave per batch slot s. Slots whose key already occurred earlier exit;
// the first occurrence sums its key's gradient rows in batch order (g[s],
// then + g[t] for each later t with the same key: the order of TF's
// unsorted_segment_sum over the deduplicated IndexedSlices) and publishes
// its slot in mark[key]. Occurrences are found 64 slots per ballot.
__global__ __launch_bounds__(64) void sparse_dedup_kernel(const int32_t* __restrict__ idx, int B, int dim,
                                                          const float* __restrict__ g, float* __restrict__ gsum,
                                                          int32_t* __restrict__ mark) {
  const int s = blockIdx.x, lane = threadIdx.x;
  const int32_t key = idx[s];
  for (int t0 = 0; t0 < s; t0 += kWave) {
    const int t = t0 + lane;
    if (__ballot(t < s && idx[t] == key)) return;  // wave-uniform: not the first occurrence
  }
  for (int c0 = 0; c0 < dim; c0 += kWave) {
    const int c = c0 + lane;
    const bool on = c < dim;
    float acc = on ? g[(int64_t)s * dim + c] : 0.f;
    for (int t0 = s + 1; t0 < B; t0 += kWave) {
      const int t = t0 + lane;
      uint64_t m = __ballot(t < B && idx[t] == key);
      while (m) {  // ascending slot order
        const int u = t0 + __builtin_ctzll(m);
        m &= m - 1;
        if (on) acc = acc + g[(int64_t)u * dim + c];
      }
    }
    if (on) gsum[(int64_t)s * dim + c] = acc;
  }
  if (lane == 0) mark[key] = s;
}

// Keras OptimizerV2 Adam._resource_apply_sparse: whole-table decay of m and
// v, scatter-add of the (deduplicated) slices, whole-table var update.
__global__ __launch_bounds__(kBlock) void adam_sparse_table_kernel(float* __restrict__ var, float* __restrict__ m,
                                                                    float* __restrict__ v, int64_t n_rows, int dim,
                                                                    const int32_t* __restrict__ mark,
                                                                    const float* __restrict__ gsum, float lr,
                                                                    float b1, float omb1, float b2, float omb2,
                                                                    float eps) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= n_rows * dim) return;
  const int64_t r = o / dim;
  const int c = (int)(o - r * dim);
  const int32_t q = mark[r];
  float mo = m[o] * b1;
  float vo = v[o] * b2;
  if (q >= 0) {
    const float gr = gsum[(int64_t)q * dim + c];
    mo = mo + gr * omb1;
    vo = vo + (gr * gr) * omb2;
  }
  m[o] = mo;
  v[o] = vo;
  var[o] = var[o] - (lr * mo) / (sqrtf(vo) + eps);
}

// The same update, 4 consecutive elements of one row per thread (dim % 4 ==
// 0): 16-B loads and stores for the whole-table sweep, identical arithmetic.
__global__ __launch_bounds__(kBlock) void adam_sparse_table4_kernel(float* __restrict__ var, float* __restrict__ m,
                                                                     float* __restrict__ v, int64_t n_rows, int dim,
                                                                     const int32_t* __restrict__ mark,
                                                                     const float* __restrict__ gsum, float lr,
                                                                     float b1, float omb1, float b2, float omb2,
                                                                     float eps) {
  const int64_t o4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o4 * 4 >= n_rows * dim) return;
  const int64_t o = o4 * 4;
  const int64_t r = o / dim;
  const int c = (int)(o - r * dim);
  const int32_t q = mark[r];
  float4 mo = reinterpret_cast<const float4*>(m)[o4];
  float4 vo = reinterpret_cast<const float4*>(v)[o4];
  float4 xo = reinterpret_cast<const float4*>(var)[o4];
  float* mp = &mo.x;
  float* vp = &vo.x;
  float* xp = &xo.x;
  float4 gr = make_float4(0.f, 0.f, 0.f, 0.f);
  if (q >= 0) gr = *reinterpret_cast<const float4*>(gsum + (int64_t)q * dim + c);
  const float* gp = &gr.x;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float me = mp[e] * b1;
    float ve = vp[e] * b2;
    if (q >= 0) {
      me = me + gp[e] * omb1;
      ve = ve + (gp[e] * gp[e]) * omb2;
    }
    mp[e] = me;
    vp[e] = ve;
    xp[e] = xp[e] - (lr * me) / (sqrtf(ve) + eps);
  }
  reinterpret_cast<float4*>(m)[o4] = mo;
  reinterpret_cast<float4*>(v)[o4] = vo;
  reinterpret_cast<float4*>(var)[o4] = xo;
}

// Grouped form (hrec_adam_sparse_tables): one launch per phase for all
// tables. Work item ranges per table are prefix sums in the kernel argument.
struct SparseGroup {
  hrec_sparse_table t[HREC_MAX_SPARSE_TABLES];
  int64_t start[HREC_MAX_SPARSE_TABLES + 1];  // first work item (slot / block) of table i
  int n;
};

__device__ __forceinline__ int group_of(const SparseGroup& G, int64_t x) {
  int i = 0;
  while (i + 1 < G.n && x >= G.start[i + 1]) ++i;
  return i;
}

// blocks of one wave: block b is slot (b - start[i]) of table i
__global__ __launch_bounds__(64) void sparse_dedup_group_kernel(const SparseGroup G) {
  const int i = group_of(G, blockIdx.x);
  const hrec_sparse_table& T = G.t[i];
  const int s = (int)(blockIdx.x - G.start[i]), lane = threadIdx.x;
  const int32_t* __restrict__ idx = T.indices;
  const float* __restrict__ g = T.grad_rows;
  const int B = T.batch, dim = T.dim;
  const int32_t key = idx[s];
  for (int t0 = 0; t0 < s; t0 += kWave) {
    const int t = t0 + lane;
    if (__ballot(t < s && idx[t] == key)) return;
  }
  for (int c0 = 0; c0 < dim; c0 += kWave) {
    const int c = c0 + lane;
    const bool on = c < dim;
    float acc = on ? g[(int64_t)s * dim + c] : 0.f;
    for (int t0 = s + 1; t0 < B; t0 += kWave) {
      const int t = t0 + lane;
      uint64_t msk = __ballot(t < B && idx[t] == key);
      while (msk) {
        const int u = t0 + __builtin_ctzll(msk);
        msk &= msk - 1;
        if (on) acc = acc + g[(int64_t)u * dim + c];
      }
    }
    if (on) T.gsum[(int64_t)s * dim + c] = acc;
  }
  if (lane == 0) T.mark[key] = s;
}

// One element of the whole-table Adam step (has_g: the row is in the batch;
// g its summed gradient). The two fma are spelled out so every kernel that
// updates a row (the sweep, the touched-rows kernel of the phased form)
// rounds it identically.
__device__ __forceinline__ void adam_elem(float& m, float& v, float& x, float g, bool has_g, float lr, float b1,
                                          float omb1, float b2, float omb2, float eps) {
  float me = m * b1;
  float ve = v * b2;
  if (has_g) {
    me = __builtin_fmaf(g, omb1, me);
    ve = __builtin_fmaf(g * g, omb2, ve);
  }
  m = me;
  v = ve;
  x = x - (lr * me) / (sqrtf(ve) + eps);
}

// blocks of kBlock threads x 4 elements (every dim % 4 == 0, 16-B aligned).
// SKIP_TOUCHED (phase 1 of the phased form): rows marked in this batch are
// left alone (phase 2 updates them once the gradients exist).
template <bool SKIP_TOUCHED>
__global__ __launch_bounds__(kBlock) void adam_sparse_group4_kernel(const SparseGroup G, float lr, float b1,
                                                                     float omb1, float b2, float omb2, float eps) {
  const int i = group_of(G, blockIdx.x);
  const hrec_sparse_table& T = G.t[i];
  const int64_t o4 = (blockIdx.x - G.start[i]) * (int64_t)kBlock + threadIdx.x;
  const int dim = T.dim;
  if (o4 * 4 >= T.n_rows * dim) return;
  const int64_t o = o4 * 4;
  const int64_t r = o / dim;
  const int c = (int)(o - r * dim);
  const int32_t q = T.mark[r];
  if (SKIP_TOUCHED && q >= 0) return;
  float4 mo = reinterpret_cast<const float4*>(T.m)[o4];
  float4 vo = reinterpret_cast<const float4*>(T.v)[o4];
  float4 xo = reinterpret_cast<const float4*>(T.var)[o4];
  float* mp = &mo.x;
  float* vp = &vo.x;
  float* xp = &xo.x;
  float4 gr = make_float4(0.f, 0.f, 0.f, 0.f);
  if (!SKIP_TOUCHED && q >= 0) gr = *reinterpret_cast<const float4*>(T.gsum + (int64_t)q * dim + c);
  const float* gp = &gr.x;
#pragma unroll
  for (int e = 0; e < 4; ++e) adam_elem(mp[e], vp[e], xp[e], gp[e], !SKIP_TOUCHED && q >= 0, lr, b1, omb1, b2, omb2, eps);
  reinterpret_cast<float4*>(T.m)[o4] = mo;
  reinterpret_cast<float4*>(T.v)[o4] = vo;
  reinterpret_cast<float4*>(T.var)[o4] = xo;
}

// Phase 0 of the phased form: mark[key] = first slot of key (no gradients).
__global__ __launch_bounds__(64) void sparse_mark_group_kernel(const SparseGroup G) {
  const int i = group_of(G, blockIdx.x);
  const hrec_sparse_table& T = G.t[i];
  const int s = (int)(blockIdx.x - G.start[i]), lane = threadIdx.x;
  const int32_t* __restrict__ idx = T.indices;
  const int32_t key = idx[s];
  for (int t0 = 0; t0 < s; t0 += kWave) {
    const int t = t0 + lane;
    if (__ballot(t < s && idx[t] == key)) return;
  }
  if (lane == 0) T.mark[key] = s;
}

// Phase 2: one wave per first slot of a key — the slots' gradients summed in
// slot order (as sparse_dedup_group_kernel) and the row's Adam step (as the
// sweep's marked rows), straight into var / m / v.
__global__ __launch_bounds__(64) void sparse_touched_group_kernel(const SparseGroup G, float lr, float b1, float omb1,
                                                                  float b2, float omb2, float eps) {
  const int i = group_of(G, blockIdx.x);
  const hrec_sparse_table& T = G.t[i];
  const int s = (int)(blockIdx.x - G.start[i]), lane = threadIdx.x;
  const int32_t* __restrict__ idx = T.indices;
  const float* __restrict__ g = T.grad_rows;
  const int B = T.batch, dim = T.dim;
  const int32_t key = idx[s];
  if (T.mark[key] != s) return;  // a later slot of a key: summed by its first
  for (int c0 = 0; c0 < dim; c0 += kWave) {
    const int c = c0 + lane;
    const bool on = c < dim;
    float acc = on ? g[(int64_t)s * dim + c] : 0.f;
    for (int t0 = s + 1; t0 < B; t0 += kWave) {
      const int t = t0 + lane;
      uint64_t msk = __ballot(t < B && idx[t] == key);
      while (msk) {
        const int u = t0 + __builtin_ctzll(msk);
        msk &= msk - 1;
        if (on) acc = acc + g[(int64_t)u * dim + c];
      }
    }
    if (on) {
      const int64_t o = (int64_t)key * dim + c;
      float m = T.m[o], v = T.v[o], x = T.var[o];
      adam_elem(m, v, x, acc, true, lr, b1, omb1, b2, omb2, eps);
      T.m[o] = m;
      T.v[o] = v;
      T.var[o] = x;
    }
  }
}

__global__ void sparse_unmark_group_kernel(const SparseGroup G) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= G.start[G.n]) return;
  const int i = group_of(G, x);
  const hrec_sparse_table& T = G.t[i];
  T.mark[T.indices[x - G.start[i]]] = -1;
}

__global__ void sparse_unmark_kernel(const int32_t* __restrict__ idx, int B, int32_t* __restrict__ mark) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < B) mark[idx[s]] = -1;
}

static TTDev to_dev(const hrec_tt_params* p) {
  TTDev t;
  t.d = p->d;
  t.ue = p->user_emb;
  t.ie = p->item_emb;
  t.me = p->man_emb;
  t.ce = p->cat_emb;
  t.w1 = p->w1;
  t.b1 = p->b1;
  t.w2 = p->w2;
  t.b2 = p->b2;
  t.gu = p->ln_user_gamma;
  t.bu = p->ln_user_beta;
  t.gi = p->ln_item_gamma;
  t.bi = p->ln_item_beta;
  return t;
}

static bool params_ok(const hrec_tt_params* p) {
  return p && p->d >= 1 && p->d <= 1024 && p->user_emb && p->item_emb && p->man_emb && p->cat_emb && p->w1 &&
         p->b1 && p->w2 && p->b2 && p->ln_user_gamma && p->ln_user_beta && p->ln_item_gamma && p->ln_item_beta;
}

}  // namespace hrec

using namespace hrec;

// the matrix-core item tower (csrc/tt_mfma.hip) for d <= 256; 1 = use the
// scalar kernel below
static int item_forward(const hrec_tt_params& p, const int32_t* item, const int32_t* man, const int32_t* cat,
                        const float* numeric, int64_t n, float* out, float* z, float* xh, float* rs, void* stream) {
  return hrec_tt_item_forward_mfma(p.d, p.item_emb, p.man_emb, p.cat_emb, p.w1, p.b1, p.w2, p.b2, p.ln_item_gamma,
                                   p.ln_item_beta, item, man, cat, numeric, n, out, z, xh, rs, stream);
}

static size_t item_fwd_smem(int d) { return (size_t)kTR * (2 * d + 32) * sizeof(float); }

extern "C" int hrec_tt_item_forward(const hrec_tt_params* params, const int32_t* item, const int32_t* manufacturer,
                                    const int32_t* category, const float* numeric, int64_t n, float* item_vec,
                                    void* stream) {
  HREC_REQUIRE(params_ok(params), "tt_item_forward: bad parameter block");
  HREC_REQUIRE(n >= 0, "tt_item_forward: negative n");
  if (n == 0) return HREC_OK;
  HREC_REQUIRE(item && manufacturer && category && numeric && item_vec, "tt_item_forward: null pointer");
  const int rc = item_forward(*params, item, manufacturer, category, numeric, n, item_vec, nullptr, nullptr, nullptr,
                              stream);
  if (rc <= 0) return rc;
  const size_t sm = item_fwd_smem(params->d);
  HREC_REQUIRE(sm <= 160 * 1024, "tt_item_forward: embedding_size too large for one LDS tile");
  hipLaunchKernelGGL(tt_item_forward_kernel, dim3((unsigned)((n + kTR - 1) / kTR)), dim3(kBlock), sm,
                     as_stream(stream), to_dev(params), item, manufacturer, category, numeric, n, item_vec,
                     nullptr, nullptr, nullptr);
  return check_launch("tt_item_forward_kernel");
}

extern "C" int hrec_tt_user_forward(const hrec_tt_params* params, const int32_t* user, int64_t n, float* user_vec,
                                    void* stream) {
  HREC_REQUIRE(params_ok(params), "tt_user_forward: bad parameter block");
  HREC_REQUIRE(n >= 0, "tt_user_forward: negative n");
  if (n == 0) return HREC_OK;
  HREC_REQUIRE(user && user_vec, "tt_user_forward: null pointer");
  hipLaunchKernelGGL(tt_user_forward_kernel, dim3((unsigned)((n + 3) / 4)), dim3(kBlock), 0, as_stream(stream),
                     to_dev(params), user, n, user_vec, nullptr, nullptr);
  return check_launch("tt_user_forward_kernel");
}

extern "C" int hrec_tt_score(const float* user_vec, int n_users, const float* item_vec, int64_t n_items, int d,
                             float* out, void* stream) {
  HREC_REQUIRE(n_users >= 0 && n_items >= 0 && d >= 1, "tt_score: bad shape");
  if (n_users == 0 || n_items == 0) return HREC_OK;
  HREC_REQUIRE(n_users < 65536, "tt_score: at most 65535 users per call");
  HREC_REQUIRE(user_vec && item_vec && out, "tt_score: null pointer");
  // widths the K8 matrix-core dot handles natively, at every batch size (its
  // GEMV for 1-4 users issues the tiles' MFMA sequence: the same bits): exact
  // f32 fma chains per k-step, item fragments kept in registers across the
  // user chunks, XCD-aware tile order (csrc/dot_topk.hip) — 0.91 of the f32
  // peak at c4 against ~0.33 for the LDS-staged tile kernel below
  const bool aligned = (((uintptr_t)user_vec | (uintptr_t)item_vec) & 15) == 0;
  if (tt_dot_order(d) && aligned)
    return hrec_dot_scores(user_vec, n_users, item_vec, n_items, d, 0, out, n_items, stream);
  if (n_users < 8 || tt_dot_order(d)) {  // GEMV-shaped (or unaligned K8 widths): one thread per (user, item)
    hipLaunchKernelGGL(tt_score_kernel, dim3((unsigned)((n_items + kBlock - 1) / kBlock), (unsigned)n_users),
                       dim3(kBlock), 0, as_stream(stream), user_vec, n_users, item_vec, n_items, d, out);
    return check_launch("tt_score_kernel");
  }
  HREC_REQUIRE((n_items + 63) / 64 < (1ll << 32), "tt_score: grid too large");
  if (HREC_TT_SCORE_V2 && d % 4 == 0 && (((uintptr_t)user_vec | (uintptr_t)item_vec) & 15) == 0) {
    hipLaunchKernelGGL(tt_score_mfma2_kernel, dim3((unsigned)((n_items + 63) / 64)), dim3(256), 0,
                       as_stream(stream), user_vec, n_users, item_vec, n_items, d, out);
    return check_launch("tt_score_mfma2_kernel");
  }
  hipLaunchKernelGGL(tt_score_mfma_kernel, dim3((unsigned)((n_items + 63) / 64)),
                     dim3(256), 0, as_stream(stream), user_vec, n_users, item_vec, n_items, d, out);
  return check_launch("tt_score_mfma_kernel");
}

static size_t partial_len(int d) { return (size_t)(d + 32) * d + 5 * (size_t)d + 48 + 2; }

extern "C" size_t hrec_tt_train_workspace_bytes(int d, int64_t batch) {
  const int64_t nblk = (batch + kTR - 1) / kTR;
  const size_t scalar_part = (size_t)nblk * partial_len(d), mfma_scratch = (size_t)batch * (d + 19);
  const size_t f = (size_t)batch * (4 * (size_t)d + (d + 32) + 2) +
                   (scalar_part > mfma_scratch ? scalar_part : mfma_scratch);
  return f * sizeof(float) + 256;
}

extern "C" size_t hrec_tt_grad_len(int d) { return partial_len(d); }

extern "C" int hrec_tt_forward_backward(const hrec_tt_params* params, const int32_t* user, const int32_t* item,
                                        const int32_t* manufacturer, const int32_t* category, const float* numeric,
                                        const float* y, int64_t batch, float* grad_dense, float* g_user,
                                        float* g_item, float* g_man, float* g_cat, void* workspace,
                                        size_t workspace_bytes, void* stream) {
  HREC_REQUIRE(params_ok(params), "tt_forward_backward: bad parameter block");
  HREC_REQUIRE(batch >= 1 && batch < (1ll << 31), "tt_forward_backward: bad batch");
  HREC_REQUIRE(user && item && manufacturer && category && numeric && y && grad_dense && g_user && g_item && g_man &&
                   g_cat && workspace,
               "tt_forward_backward: null pointer");
  const int d = params->d;
  const size_t need = hrec_tt_train_workspace_bytes(d, batch);
  HREC_REQUIRE(workspace_bytes >= need, "tt_forward_backward: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t s = as_stream(stream);
  const TTDev P = to_dev(params);
  float* w = (float*)workspace;
  float* uvec = w;
  float* uxh = uvec + batch * d;
  float* ivec = uxh + batch * d;
  float* ixh = ivec + batch * d;
  float* zs = ixh + batch * d;
  float* urs = zs + batch * (d + 32);
  float* irs = urs + batch;
  float* part = irs + batch;
  const int nblk = (int)((batch + kTR - 1) / kTR);
  hipLaunchKernelGGL(tt_user_forward_kernel, dim3((unsigned)((batch + 3) / 4)), dim3(kBlock), 0, s, P, user, batch,
                     uvec, uxh, urs);
  int rc = check_launch("tt_user_forward_kernel");
  if (rc) return rc;
  rc = item_forward(*params, item, manufacturer, category, numeric, batch, ivec, zs, ixh, irs, stream);
  if (rc < 0) return rc;
  if (rc == 1) {
    hipLaunchKernelGGL(tt_item_forward_kernel, dim3((unsigned)nblk), dim3(kBlock), item_fwd_smem(d), s, P, item,
                       manufacturer, category, numeric, batch, ivec, zs, ixh, irs);
    rc = check_launch("tt_item_forward_kernel");
    if (rc) return rc;
  }
  // backward with both Dense GEMMs on the matrix cores (csrc/tt_mfma.hip);
  // the scratch (B·(d + 19) floats) reuses the partials region
  rc = hrec_tt_backward_mfma(d, P.w2, P.gu, P.gi, y, batch, uvec, uxh, urs, ivec, ixh, irs, zs, numeric, g_user,
                             g_item, g_man, g_cat, grad_dense, part, stream);
  if (rc <= 0) return rc;  // 1: d needs the scalar kernels below
  const size_t bsm = ((size_t)kTR * d + kTR * 16 + kTR + 8) * sizeof(float);
  hipLaunchKernelGGL(tt_backward_kernel, dim3((unsigned)nblk), dim3(kBlock), bsm, s, P, y, batch, uvec, uxh, urs,
                     ivec, ixh, irs, zs, numeric, g_user, g_item, g_man, g_cat, part);
  rc = check_launch("tt_backward_kernel");
  if (rc) return rc;
  const size_t plen = partial_len(d);
  hipLaunchKernelGGL(tt_reduce_partials_kernel, dim3((unsigned)((plen + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                     part, nblk, plen, grad_dense);
  return check_launch("tt_reduce_partials_kernel");
}

extern "C" int hrec_adam_dense(float* var, float* m, float* v, const float* grad, int64_t n, float alpha,
                               float beta1, float beta2, float epsilon, void* stream) {
  HREC_REQUIRE(n >= 0, "adam_dense: negative n");
  if (n == 0) return HREC_OK;
  HREC_REQUIRE(var && m && v && grad, "adam_dense: null pointer");
  hipLaunchKernelGGL(adam_dense_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     as_stream(stream), var, m, v, grad, n, alpha, beta1, beta2, epsilon);
  return check_launch("adam_dense_kernel");
}

extern "C" int hrec_adam_sparse(float* var, float* m, float* v, int64_t n_rows, int dim, const int32_t* indices,
                                const float* grad_rows, int batch, int32_t* mark, float* gsum, float lr, float beta1,
                                float one_minus_beta1, float beta2, float one_minus_beta2, float epsilon,
                                void* stream) {
  HREC_REQUIRE(n_rows >= 0 && dim >= 1 && batch >= 0, "adam_sparse: bad shape");
  if (n_rows == 0) return HREC_OK;
  HREC_REQUIRE(var && m && v && mark, "adam_sparse: null pointer");
  HREC_REQUIRE(batch == 0 || (indices && grad_rows && gsum), "adam_sparse: null slices");
  hipStream_t s = as_stream(stream);
  if (batch > 0) {
    hipLaunchKernelGGL(sparse_dedup_kernel, dim3((unsigned)batch), dim3(kWave), 0, s, indices, batch, dim, grad_rows,
                       gsum, mark);
    int rc = check_launch("sparse_dedup_kernel");
    if (rc) return rc;
  }
  const int64_t total = n_rows * dim;
  const bool vec4 = dim % 4 == 0 && (((uintptr_t)var | (uintptr_t)m | (uintptr_t)v | (uintptr_t)gsum) & 15) == 0;
  if (vec4) {
    hipLaunchKernelGGL(adam_sparse_table4_kernel, dim3((unsigned)((total / 4 + kBlock - 1) / kBlock)), dim3(kBlock),
                       0, s, var, m, v, n_rows, dim, mark, gsum, lr, beta1, one_minus_beta1, beta2, one_minus_beta2,
                       epsilon);
  } else {
    hipLaunchKernelGGL(adam_sparse_table_kernel, dim3((unsigned)((total + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                       var, m, v, n_rows, dim, mark, gsum, lr, beta1, one_minus_beta1, beta2, one_minus_beta2,
                       epsilon);
  }
  int rc = check_launch("adam_sparse_table_kernel");
  if (rc || batch == 0) return rc;
  hipLaunchKernelGGL(sparse_unmark_kernel, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0, s, indices, batch,
                     mark);
  return check_launch("sparse_unmark_kernel");
}

extern "C" int hrec_adam_sparse_tables(const hrec_sparse_table* tables, int n_tables, float lr, float beta1,
                                       float one_minus_beta1, float beta2, float one_minus_beta2, float epsilon,
                                       void* stream) {
  HREC_REQUIRE(n_tables >= 0 && n_tables <= HREC_MAX_SPARSE_TABLES, "adam_sparse_tables: 0..%d tables",
               HREC_MAX_SPARSE_TABLES);
  if (n_tables == 0) return HREC_OK;
  HREC_REQUIRE(tables, "adam_sparse_tables: null table list");
  bool vec4 = true;
  for (int i = 0; i < n_tables; ++i) {
    const hrec_sparse_table& T = tables[i];
    HREC_REQUIRE(T.n_rows >= 0 && T.dim >= 1 && T.batch >= 0, "adam_sparse_tables: table %d: bad shape", i);
    HREC_REQUIRE(T.n_rows == 0 || (T.var && T.m && T.v && T.mark), "adam_sparse_tables: table %d: null pointer", i);
    HREC_REQUIRE(T.batch == 0 || (T.indices && T.grad_rows && T.gsum),
                 "adam_sparse_tables: table %d: null slices", i);
    vec4 = vec4 && T.dim % 4 == 0 &&
           (((uintptr_t)T.var | (uintptr_t)T.m | (uintptr_t)T.v | (uintptr_t)T.gsum) & 15) == 0;
  }
  hipStream_t s = as_stream(stream);
  if (!vec4) {  // per table (rare shapes: d % 4 != 0)
    for (int i = 0; i < n_tables; ++i) {
      const hrec_sparse_table& T = tables[i];
      const int rc = hrec_adam_sparse(T.var, T.m, T.v, T.n_rows, T.dim, T.indices, T.grad_rows, T.batch, T.mark,
                                      T.gsum, lr, beta1, one_minus_beta1, beta2, one_minus_beta2, epsilon, stream);
      if (rc) return rc;
    }
    return HREC_OK;
  }
  SparseGroup G{};
  // phase 1: slots; tables with no rows keep their (empty) batch out
  G.n = 0;
  int64_t acc = 0;
  for (int i = 0; i < n_tables; ++i) {
    if (tables[i].n_rows == 0) continue;
    G.t[G.n] = tables[i];
    G.start[G.n] = acc;
    acc += tables[i].batch;
    ++G.n;
  }
  G.start[G.n] = acc;
  if (G.n == 0) return HREC_OK;
  const int64_t n_slots = acc;
  if (n_slots > 0) {
    hipLaunchKernelGGL(sparse_dedup_group_kernel, dim3((unsigned)n_slots), dim3(kWave), 0, s, G);
    const int rc = check_launch("sparse_dedup_group_kernel");
    if (rc) return rc;
  }
  // phase 2: whole-table sweeps, each table starting on a block boundary
  SparseGroup H = G;
  acc = 0;
  for (int i = 0; i < H.n; ++i) {
    H.start[i] = acc;
    acc += (H.t[i].n_rows * H.t[i].dim / 4 + kBlock - 1) / kBlock;
  }
  H.start[H.n] = acc;
  hipLaunchKernelGGL(adam_sparse_group4_kernel<false>, dim3((unsigned)acc), dim3(kBlock), 0, s, H, lr, beta1,
                     one_minus_beta1, beta2, one_minus_beta2, epsilon);
  int rc = check_launch("adam_sparse_group4_kernel");
  if (rc || n_slots == 0) return rc;
  // phase 3: restore mark = -1
  hipLaunchKernelGGL(sparse_unmark_group_kernel, dim3((unsigned)((n_slots + 255) / 256)), dim3(256), 0, s, G);
  return check_launch("sparse_unmark_group_kernel");
}

extern "C" int hrec_tt_pair_score(const float* user_vec, const float* item_vec, int64_t n, int d, float* out,
                                  void* stream) {
  HREC_REQUIRE(n >= 0 && d >= 1, "tt_pair_score: bad shape");
  if (n == 0) return HREC_OK;
  HREC_REQUIRE(user_vec && item_vec && out, "tt_pair_score: null pointer");
  hipLaunchKernelGGL(tt_pair_score_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, as_stream(stream),
                     user_vec, item_vec, n, d, out);
  return check_launch("tt_pair_score_kernel");
}

// hrec_adam_sparse_tables split into phases (HREC_SPARSE_*), so that the
// whole-table sweep of the rows the batch does not touch — nearly all of the
// step's HBM traffic — can run on a second stream beside the batch's
// forward / backward (which read only touched rows). Phases 0, 1, 2, 3 in
// stream order give bit for bit the rows of hrec_adam_sparse_tables; phase 1
// may overlap phase 2 (disjoint rows) but neither phase 0 nor phase 3 (they
// write the marks phase 1 reads). Needs dim % 4 == 0 and 16-B aligned
// var / m / v (hrec_adam_sparse_tables takes every shape); gsum is unused and
// grad_rows is read by phase 2 only.
extern "C" int hrec_adam_sparse_tables_phase(const hrec_sparse_table* tables, int n_tables, int phase, float lr,
                                             float beta1, float one_minus_beta1, float beta2, float one_minus_beta2,
                                             float epsilon, void* stream) {
  HREC_REQUIRE(n_tables >= 0 && n_tables <= HREC_MAX_SPARSE_TABLES, "adam_sparse_tables_phase: 0..%d tables",
               HREC_MAX_SPARSE_TABLES);
  HREC_REQUIRE(phase >= HREC_SPARSE_MARK && phase <= HREC_SPARSE_UNMARK, "adam_sparse_tables_phase: phase %d not in 0..3",
               phase);
  if (n_tables == 0) return HREC_OK;
  HREC_REQUIRE(tables, "adam_sparse_tables_phase: null table list");
  for (int i = 0; i < n_tables; ++i) {
    const hrec_sparse_table& T = tables[i];
    HREC_REQUIRE(T.n_rows >= 0 && T.dim >= 1 && T.batch >= 0, "adam_sparse_tables_phase: table %d: bad shape", i);
    HREC_REQUIRE(T.n_rows == 0 || (T.var && T.m && T.v && T.mark), "adam_sparse_tables_phase: table %d: null pointer",
                 i);
    HREC_REQUIRE(T.batch == 0 || (T.indices && (phase != HREC_SPARSE_TOUCHED || T.grad_rows)),
                 "adam_sparse_tables_phase: table %d: null slices", i);
    HREC_REQUIRE(T.dim % 4 == 0 && (((uintptr_t)T.var | (uintptr_t)T.m | (uintptr_t)T.v) & 15) == 0,
                 "adam_sparse_tables_phase: table %d: needs dim %% 4 == 0 and 16-B aligned rows "
                 "(use hrec_adam_sparse_tables)", i);
  }
  hipStream_t s = as_stream(stream);
  SparseGroup G{};
  int64_t acc = 0;
  for (int i = 0; i < n_tables; ++i) {
    if (tables[i].n_rows == 0) continue;
    G.t[G.n] = tables[i];
    G.start[G.n] = acc;
    acc += phase == HREC_SPARSE_SWEEP_UNTOUCHED ? (tables[i].n_rows * tables[i].dim / 4 + kBlock - 1) / kBlock
                                                : tables[i].batch;
    ++G.n;
  }
  G.start[G.n] = acc;
  if (G.n == 0 || acc == 0) return HREC_OK;
  switch (phase) {
    case HREC_SPARSE_MARK:
      hipLaunchKernelGGL(sparse_mark_group_kernel, dim3((unsigned)acc), dim3(kWave), 0, s, G);
      return check_launch("sparse_mark_group_kernel");
    case HREC_SPARSE_SWEEP_UNTOUCHED:
      hipLaunchKernelGGL(adam_sparse_group4_kernel<true>, dim3((unsigned)acc), dim3(kBlock), 0, s, G, lr, beta1,
                         one_minus_beta1, beta2, one_minus_beta2, epsilon);
      return check_launch("adam_sparse_group4_kernel (untouched rows)");
    case HREC_SPARSE_TOUCHED:
      hipLaunchKernelGGL(sparse_touched_group_kernel, dim3((unsigned)acc), dim3(kWave), 0, s, G, lr, beta1,
                         one_minus_beta1, beta2, one_minus_beta2, epsilon);
      return check_launch("sparse_touched_group_kernel");
    default:
      hipLaunchKernelGGL(sparse_unmark_group_kernel, dim3((unsigned)((acc + 255) / 256)), dim3(256), 0, s, G);
      return check_launch("sparse_unmark_group_kernel");
  }
}
