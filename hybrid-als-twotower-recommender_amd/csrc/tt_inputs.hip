// K4i: the two-tower item inputs of one predict_for_user call, built on the
// device from the candidate frame's raw columns (src/two_tower_model.py:136-146:
// the item_id_in / manufacturer_in / category_in columns as Keras float32
// Inputs cast to int32 by the Embeddings, numeric_in =
// scaler.transform(frame[["price", "average_review_rating"]])). The host
// used to make five numpy passes per id column (f32 round trip, range check,
// int32 cast) and a pandas sub-frame copy for the scaler; here one pass over
// the uploaded int64 / f64 columns does all of it:
//   ids: v in [0, table) and |v| < 2^24 (where the f32 round trip is the
//        identity) -> int32; anything else raises kHrecInputsIds and the
//        caller redoes the call on the host (the reference's error or cast);
//   numeric: x * scale_ + min_ in f64, rounded once to f32 (sklearn's
//        X *= scale_; X += min_ then np.asarray(dtype=float32); separate
//        rounded operations: contraction off); an infinite input raises
//        kHrecInputsInf (sklearn's own validation error on the host);
//   duplicates: a per-call presence bitmap over the item table (atomicOr on
//        a bit already set raises kHrecInputsDup: the hybrid's array path
//        needs unique candidate ids).
// Integer and byte work, HBM-bound: 40 B read + 20 B written per row.
#include "common.h"

namespace hrec {

constexpr int kHrecInputsIds = 1;
constexpr int kHrecInputsInf = 2;
constexpr int kHrecInputsDup = 4;

__device__ __forceinline__ bool ti_ok(int64_t v, int64_t table) {
  return v >= 0 && v < table && v < (1ll << 24);
}

__global__ __launch_bounds__(256) void tt_item_inputs_kernel(
    const int64_t* __restrict__ item, const int64_t* __restrict__ man, const int64_t* __restrict__ cat,
    const double* __restrict__ price, const double* __restrict__ rating, int64_t n, int64_t n_item, int64_t n_man,
    int64_t n_cat, double s0, double m0, double s1, double m1, int32_t* __restrict__ item_out,
    int32_t* __restrict__ man_out, int32_t* __restrict__ cat_out, float* __restrict__ numeric_out,
    uint32_t* __restrict__ seen, int32_t* __restrict__ flags) {
#pragma clang fp contract(off)
  int bad = 0;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = item[r], b = man[r], c = cat[r];
    const double p = price[r], q = rating[r];
    const bool ok = ti_ok(a, n_item) && ti_ok(b, n_man) && ti_ok(c, n_cat);
    bad |= ok ? 0 : kHrecInputsIds;
    item_out[r] = ok ? (int32_t)a : 0;
    man_out[r] = ok ? (int32_t)b : 0;
    cat_out[r] = ok ? (int32_t)c : 0;
    bad |= (isinf(p) || isinf(q)) ? kHrecInputsInf : 0;
    double x0 = p * s0;
    x0 = x0 + m0;
    double x1 = q * s1;
    x1 = x1 + m1;
    reinterpret_cast<float2*>(numeric_out)[r] = make_float2((float)x0, (float)x1);
    if (ok) {
      const uint32_t bit = 1u << (a & 31);
      if (atomicOr(&seen[a >> 5], bit) & bit) bad |= kHrecInputsDup;
    }
  }
  // one flag update per wave
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) bad |= __shfl_xor(bad, off, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicOr(flags, bad);
}

}  // namespace hrec

using namespace hrec;

extern "C" size_t hrec_tt_item_inputs_workspace_bytes(int64_t n_item_table) {
  return 16 + (size_t)((n_item_table > 0 ? n_item_table : 0) + 31) / 32 * 4;
}

extern "C" int hrec_tt_item_inputs(const int64_t* item, const int64_t* manufacturer, const int64_t* category,
                                   const double* price, const double* rating, int64_t n, int64_t n_item_table,
                                   int64_t n_man_table, int64_t n_cat_table, const double* scale, const double* min_,
                                   int32_t* item_out, int32_t* man_out, int32_t* cat_out, float* numeric_out,
                                   int32_t* flags, void* workspace, size_t workspace_bytes, void* stream) {
  HREC_REQUIRE(n >= 0 && n_item_table >= 0 && n_man_table >= 0 && n_cat_table >= 0, "tt_item_inputs: bad sizes");
  HREC_REQUIRE(scale && min_ && flags, "tt_item_inputs: null scale / min / flags");
  const size_t need = hrec_tt_item_inputs_workspace_bytes(n_item_table);
  HREC_REQUIRE(workspace && workspace_bytes >= need, "tt_item_inputs: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t s = as_stream(stream);
  // flags (first 4 B of the caller's flags word) and the presence bitmap: one memset each
  if (hipMemsetAsync(flags, 0, 4, s) != hipSuccess) return check_launch("tt_item_inputs: memset");
  uint32_t* seen = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + 16);
  if (hipMemsetAsync(seen, 0, need - 16, s) != hipSuccess) return check_launch("tt_item_inputs: memset");
  if (n == 0) return HREC_OK;
  HREC_REQUIRE(item && manufacturer && category && price && rating && item_out && man_out && cat_out && numeric_out,
               "tt_item_inputs: null column");
  HREC_REQUIRE(((uintptr_t)numeric_out & 7) == 0, "tt_item_inputs: numeric_out must be 8-B aligned");
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(tt_item_inputs_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s, item,
                     manufacturer, category, price, rating, n, n_item_table, n_man_table, n_cat_table, scale[0],
                     min_[0], scale[1], min_[1], item_out, man_out, cat_out, numeric_out, seen, flags);
  return check_launch("tt_item_inputs_kernel");
}
