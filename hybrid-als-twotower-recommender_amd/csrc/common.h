// Shared helpers for the libhrec HIP sources (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/hrec.h"

namespace hrec {

// Thread-local message of the last failure (hrec_last_error()).
void set_error(const char* fmt, ...);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// After a launch: map the HIP status to an HREC code.
int check_launch(const char* what);

constexpr int kWave = 64;

// Leading dimensions of factor matrices: 16/32/64 (one wave per row in the
// half-sweep) and 96/128/192/256 (one workgroup per row, csrc/als_wide.hip).
inline bool hrec_factor_ld_ok(int kp) {
  return kp == 16 || kp == 32 || kp == 64 || kp == 96 || kp == 128 || kp == 192 || kp == 256;
}

// idx[i] += off for every id >= 0 (item-shard offsets; csrc/dot_topk.hip).
int offset_ids(int64_t* idx, int64_t n, int64_t off, hipStream_t s);

// Stable descending top-k of n_rows rows (score.hip): larger first, equal
// values -> smaller original index first (src_idx maps positions to original
// indices; entries with index -1 are skipped; row_n, if given, bounds row r
// to its first min(n, row_n[r]) entries). Workspace: topk_ws_bytes.
size_t topk_ws_bytes(int64_t n_rows, int64_t n, int kk, size_t elem);
// gate (optional): a device flag; the launches do nothing while *gate == 0
// (a device-side fallback that needs no host round trip).
template <typename T>
int topk_rows(const T* vals, int64_t n_rows, int64_t n, int64_t row_stride, int kk, int64_t* out_idx,
              T* out_val, void* ws, size_t ws_bytes, hipStream_t s, const int64_t* src_idx = nullptr,
              const int* row_n = nullptr, const int* gate = nullptr);

// Stable descending top-k by a full per-row radix sort (csrc/sort_topk.hip),
// for top_k above the selection kernels' 1024; rows * n < 2^31.
size_t sort_topk_ws_bytes(int64_t n_rows, int64_t n);
template <typename T>
int sort_topk_rows(const T* vals, int64_t n_rows, int64_t n, int64_t row_stride, int kk, int64_t* out_idx,
                   T* out_val, void* ws, size_t ws_bytes, hipStream_t s);

// Buffer resource over rows [row0, n_rows) of a row-major matrix of
// row_bytes (< 2^14) per row, for structured loads (vindex = row - row0).
// The hardware forms vindex * stride + voffset as a 32-bit offset, which
// wraps at 4 GiB, so a resource never spans more than that: streaming
// kernels re-base it per tile (rows past the span read as zeros, like rows
// past the end of the matrix).
typedef int hrec_rsrc_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ hrec_rsrc_t rows_rsrc(const void* base, int64_t row0, int row_bytes, int64_t n_rows) {
  const uint64_t a = (uint64_t)base + (uint64_t)row0 * (uint64_t)row_bytes;
  const int64_t span = (int64_t)(0xffffffffull / (uint64_t)row_bytes);
  int64_t rem = n_rows - row0;
  rem = rem < 0 ? 0 : (rem > span ? span : rem);
  hrec_rsrc_t r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32) | (row_bytes << 16));
  r.z = __builtin_amdgcn_readfirstlane((int)(uint32_t)rem);
  r.w = 0x00020000;
  return r;
}

// Allow a kernel the CU's whole LDS (160 KiB) as dynamic shared memory, once
// per kernel (hipFuncSetAttribute costs a runtime call per launch otherwise).
bool allow_max_lds_ptr(const void* kfn);  // csrc/capi.hip: a set of the kernels already raised
template <typename K>
inline bool allow_max_lds(K kfn) {
  return allow_max_lds_ptr((const void*)kfn);
}

// splitmix64 finaliser; host and device identical (integer only).
__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// h64(seed, u, i) of BASELINE.md §3 (u, i < 2^32).
__host__ __device__ inline uint64_t pair_hash(uint64_t seed, uint64_t u, uint64_t i) {
  return mix64(seed * 0x9E3779B97F4A7C15ull + ((u << 32) | (i & 0xffffffffull)));
}

}  // namespace hrec

// csrc/als_wide.hip: the half-sweep for kp in {96, 128, 192, 256} (arguments
// already validated by hrec_als_half_sweep).
int hrec_als_half_sweep_wide(const int64_t* indptr, const int32_t* indices, const float* values, int64_t n_rows,
                             const float* src_factors, int64_t n_src, int k, int kp, double reg_param,
                             float* dst_factors, void* stream);

// csrc/tt_mfma.hip: the item tower on the f32 matrix cores for d <= 256
// (returns 1 when d needs the scalar kernel of csrc/tt.hip instead).
int hrec_tt_item_forward_mfma(int d, const float* ie, const float* me, const float* ce, const float* w1,
                              const float* b1, const float* w2, const float* b2, const float* gamma,
                              const float* beta, const int32_t* item, const int32_t* man, const int32_t* cat,
                              const float* numeric, int64_t n, float* out, float* z_save, float* xhat_save,
                              float* rstd_save, void* stream);

// csrc/tt_mfma.hip: the train step's backward with both Dense GEMMs on the
// f32 matrix cores (returns 1 when d needs the scalar kernels instead).
// scratch: B·(d + 19) floats.
int hrec_tt_backward_mfma(int d, const float* w2, const float* gamma_u, const float* gamma_i, const float* y,
                          int64_t B, const float* uvec, const float* uxhat, const float* urstd, const float* ivec,
                          const float* ixhat, const float* irstd, const float* zsave, const float* numeric,
                          float* g_user, float* g_item, float* g_man, float* g_cat, float* grad, float* scratch,
                          void* stream);

namespace hrec {
// csrc/hybrid_scores.hip: the bf16 hybrid score launch in one of its modes
// (0 = scores + per-row min / max, 1 = min / max + per-block max slice, no
// stores, 2 = the heavy model's survivors of per-(user, item group) bounds:
// filt) and its item-group count. uop: pre-converted bf16 user rows to stage
// as is.
struct HsFilter {
  const float* theta;  // [B][G] bounds (+inf: nothing of the group, NaN: every score)
  int hm;              // the heavy model (0 = ALS, 1 = two-tower)
  int cap;
  float* cv;
  int64_t* ci;
  int* cn;             // zeroed by the caller
};
int hybrid_scores_run(int mode, const float* als_users, int64_t als_ld, const int64_t* als_rows, int64_t n_als_rows,
                      int als_width, const float* tt_users, int64_t tt_ld, int tt_width, int n_users,
                      const void* als_items, const void* tt_items, int64_t n_items, int dk, float* als_out,
                      float* tt_out, int64_t ld_out, float* als_mm, float* tt_mm, float* part, int* argpos,
                      hipStream_t s, const uint16_t* uop = nullptr, const HsFilter* filt = nullptr);
int hs_groups(int64_t n_items);
int hs_slice_tiles(int dk);  // item tiles of 16 per wave slice (a slice = 16 * tiles items)
// csrc/dot_topk.hip: the matrix-core survivor filter (score >= thr[b]) and
// the list-overflow flag (cn[b] > cap -> *flag = 1).
int dot_filter_run(const void* U, int B, const void* V, int64_t n_items, int dk, int bf16, const float* thr,
                   int thr_stride, int64_t thr_per, int cap, float* cv, int64_t* ci, int* cn, hipStream_t s);
// the resident-user scores with at most ub_cap users per block (more blocks)
int dot_scores_run(const void* U, int B, const void* V, int64_t n_items, int dk, int bf16, float* out, int64_t ldo,
                   hipStream_t s, int ub_cap = 0);
int count_overflow(const int* cn, int n_users, int cap, int* flag, hipStream_t s);
// csrc/dot_gemv.hip: the few-user (B <= 4, f32) streaming scoring kernel, same
// contract and same score bits as the matrix-core launch of csrc/dot_topk.hip
// (FILTER: the per-user survivor filter, thr_per == 0).
bool dot_gemv_applies(int B, int64_t step, int dk, int bf16);
template <bool FILTER>
int dot_gemv_run(const void* U, int B, const void* V, int64_t n_rows, int64_t n_items, int64_t step, int dk, int bf16,
                 float* out,
                 int64_t ldo, const float* thr, int thr_stride, int cap, float* cv, int64_t* ci, int* cn, int64_t off,
                 hipStream_t s);
// csrc/scan.hip: inclusive / exclusive prefix sums (any n; workspace
// scan_ws_bytes(n)) and the extremes of an int64 column (out[0] = min,
// out[1] = max, device).
size_t scan_ws_bytes(int64_t n);
template <typename T>
int scan_run(const T* in, T* out, int64_t n, bool exclusive, void* ws, hipStream_t s);
int minmax_i64_run(const int64_t* x, int64_t n, int64_t* out, hipStream_t s);
// csrc/ingest.hip: the in-tree stable LSD radix sort of 32-bit keys (the low
// `bits` bits) carrying two 32-bit payload words, n < 2^31; workspace
// radix_pairs_ws_bytes(n) at any key width. *keys_sorted points into ws.
size_t radix_pairs_ws_bytes(int64_t n);
int radix_pairs_sort(const uint32_t* keys, const uint32_t* p0, const uint32_t* p1, int64_t n, int bits, void* ws,
                     uint32_t* p0_out, uint32_t* p1_out, const uint32_t** keys_sorted, hipStream_t s);
// csrc/score.hip: hrec_fuse_rows_topk's exact segment path, gated on *gate.
size_t fuse_rows_exact_ws_bytes(int64_t n_rows, int64_t n, int kk);
int fuse_rows_exact(const float* als, const float* tt, int64_t n_rows, int64_t n, int64_t ld, const float* als_mm,
                    const float* tt_mm, double w0, double w1, int kk, int64_t* out_idx, double* out_val, void* ws,
                    hipStream_t s, const int* gate);
}  // namespace hrec

#define HREC_REQUIRE(cond, ...)          \
  do {                                   \
    if (!(cond)) {                       \
      ::hrec::set_error(__VA_ARGS__);    \
      return HREC_E_INVALID;             \
    }                                    \
  } while (0)
