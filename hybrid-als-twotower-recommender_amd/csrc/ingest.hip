// Ingest: ratings as COO columns -> the CSR / CSC the
// half-sweep consumes, on the device.
//
// Replaces the reference's hand-over of a pandas DataFrame to Spark
// (src/als_model.py:51-62: createDataFrame + ALS.fit, which keys factors by the
// integer user / item ids and keeps duplicate (user, item) ratings as separate
// terms of the normal equations). Two steps:
//   hrec_encode_ids  : int64 ids -> sorted distinct ids + a dense int32 code per
//                      entry (numpy.unique(ids, return_inverse=True)); with the
//                      id range [lo, hi] known (hrec_minmax_i64) a range below
//                      2^31 sorts 32-bit keys on only the bits it spans;
//   hrec_coo_to_csr  : (row code, col code, rating) -> indptr / indices / values,
//                      rows ascending, entries of a row in input order
//                      (numpy.argsort(rows, kind="stable")).
// encode_ids: a marked table + scan for dense id ranges (hipCUB radix sort of
// (id, position) otherwise); coo_to_csr: a hand-written stable LSD radix sort
// of the dense row codes (below); plus O(n) integer passes. HBM-bound.

#include "common.h"

namespace hrec {

__global__ __launch_bounds__(256) void iota_i32_kernel(int32_t* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (int32_t)i;
}

// keys32[i] = ids[i] - lo as 32 unsigned bits (caller guarantees lo <= ids <= hi,
// hi - lo < 2^32)
__global__ __launch_bounds__(256) void shift_keys_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t lo,
                                                         int32_t* __restrict__ keys32) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    keys32[i] = (int32_t)(ids[i] - lo);
}

// flag[i] = 1 where sorted key i starts a new distinct value
template <typename K>
__global__ __launch_bounds__(256) void distinct_flags_kernel(const K* __restrict__ keys, int64_t n,
                                                             int32_t* __restrict__ flag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    flag[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}

// codes[pos[i]] = rank of sorted key i among the distinct keys; the first
// occurrence of each distinct key writes it (+ lo) to uniq; the last thread
// writes the distinct count.
template <typename K>
__global__ __launch_bounds__(256) void scatter_codes_kernel(const K* __restrict__ keys, int64_t lo,
                                                            const int32_t* __restrict__ pos,
                                                            const int32_t* __restrict__ flag,
                                                            const int32_t* __restrict__ incl, int64_t n,
                                                            int32_t* __restrict__ codes, int64_t* __restrict__ uniq,
                                                            int64_t* __restrict__ n_uniq) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t c = incl[i] - 1;
    codes[pos[i]] = c;
    if (flag[i]) uniq[c] = (sizeof(K) == 4 ? (int64_t)(uint32_t)keys[i] : (int64_t)keys[i]) + lo;
    if (i == n - 1) *n_uniq = (int64_t)incl[i];
  }
}

// Dense id ranges (span <= n): np.unique(return_inverse) without a sort.
// Mark the ids present in a span-long table, one inclusive scan gives every
// present id its rank among the sorted distinct ids, and the codes are read
// back from the table: two streaming passes over the ids instead of a radix
// sort of (id, position) pairs. Same codes and uniq as the sort path.
// Streaming passes take 4 independent elements per thread per iteration
// (loads in flight), grid-stride.
constexpr int kStreamUnroll = 4;

__device__ __forceinline__ void load_id_pair(const int64_t* __restrict__ ids, int64_t n, int64_t p, int64_t lo,
                                             bool vec, int64_t& a, int64_t& b) {
  // ids 2p, 2p + 1 (one 16-B load when both exist and ids is 16-B aligned),
  // shifted by lo; -1 past the end
  if (vec && 2 * p + 1 < n) {
    const longlong2 v = *reinterpret_cast<const longlong2*>(ids + 2 * p);
    a = v.x - lo;
    b = v.y - lo;
  } else {
    a = 2 * p < n ? ids[2 * p] - lo : -1;
    b = 2 * p + 1 < n ? ids[2 * p + 1] - lo : -1;
  }
}

// The input order, read by the marking passes for free: 1 when ids[2p] >
// ids[2p + 1] or ids[2p + 1] > ids[2p + 2] (a = ids[2p] - lo, b = ids[2p + 1]
// - lo; ids[2p + 2] is the lane above's a — lanes hold consecutive pairs — or,
// on the wave's last lane, a load). The caller ORs the waves' results into
// *desc: ids non-decreasing <=> codes non-decreasing (the code map is monotone).
__device__ __forceinline__ bool pair_descends(int64_t n, int64_t p, int64_t a, int64_t b, int64_t above_a,
                                              int64_t edge, int64_t lo) {
  bool d = 2 * p + 1 < n && a > b;
  if (2 * p + 2 < n) d |= b > (((threadIdx.x & 63) < 63) ? above_a : edge - lo);
  return d;
}
// x of the lane above (DPP wave_shl:1 — VALU moves, no LDS traffic beside
// the marking pass's LDS atomics); lane 63 keeps its own
__device__ __forceinline__ int64_t from_lane_above(int64_t x) {
  const int lo = __builtin_amdgcn_update_dpp((int)x, (int)x, 0x130, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(x >> 32), (int)(x >> 32), 0x130, 0xf, 0xf, false);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// ids[2p + 2] of the wave's last lane (p = lane 0's p + 63), a wave-uniform
// address: a scalar load beside the pair loads (no vector memory instruction
// for one lane), 0 past the end
__device__ __forceinline__ int64_t edge_id(const int64_t* __restrict__ ids, int64_t n, int64_t p, bool want) {
  const int64_t q = 2 * ((int64_t)__builtin_amdgcn_readfirstlane((int)(p & 0xffffffff)) |
                         ((int64_t)__builtin_amdgcn_readfirstlane((int)(p >> 32)) << 32)) + 2 * 63 + 2;
  return (want && q < n) ? ids[q] : 0;
}

// x of the lane below (DPP wave_shr:1); lane 0 keeps its own
__device__ __forceinline__ int32_t from_lane_below(int32_t x) {
  return __builtin_amdgcn_update_dpp(x, x, 0x138, 0xf, 0xf, false);
}
// Row starts of codes in input order (the code kernels, when the ids are
// non-decreasing: a CSR with rows = codes needs no pass over the codes).
// Pair p holds codes a (position 2p), b (2p + 1); prev = the code at 2p - 1
// (-1 at the start). Codes of sorted ids are dense and non-decreasing, so the
// first position of every code gets written, and the last entry closes the
// array: starts[n_uniq] = n.
__device__ __forceinline__ void pair_starts(int64_t n, int64_t p, int32_t a, int32_t b, int32_t prev,
                                            int64_t* __restrict__ starts) {
  if (a >= 0 && a != prev) starts[a] = 2 * p;
  if (2 * p + 1 < n) {
    if (b >= 0 && b != a) starts[b] = 2 * p + 1;
    if (2 * p + 2 == n && b >= 0) starts[b + 1] = n;
  } else if (a >= 0) {
    starts[a + 1] = n;  // 2p = n - 1
  }
}
// the lane-0 position before pair p (wave-uniform: p of lane 0 - 1 ... as 2p - 1)
__device__ __forceinline__ int64_t wave_prev_pos(int64_t p) {
  return 2 * ((int64_t)__builtin_amdgcn_readfirstlane((int)(p & 0xffffffff)) |
              ((int64_t)__builtin_amdgcn_readfirstlane((int)(p >> 32)) << 32)) - 1;
}

__global__ __launch_bounds__(256) void mark_present_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t lo,
                                                           int64_t span, int32_t* __restrict__ present,
                                                           int32_t* __restrict__ desc) {
  const bool vec = ((uintptr_t)ids & 15) == 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x, np = (n + 1) / 2;
  bool dsc = false, found = false;
  for (int64_t p0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p0 < np; p0 += 2 * stride) {
    int64_t v[4];
    load_id_pair(ids, n, p0, lo, vec, v[0], v[1]);
    if (p0 + stride < np) {
      load_id_pair(ids, n, p0 + stride, lo, vec, v[2], v[3]);
    } else {
      v[2] = v[3] = -1;
    }
    const int64_t e0 = edge_id(ids, n, p0, desc && !found), e2 = edge_id(ids, n, p0 + stride, desc && !found);
    if (desc && !found) {  // a wave stops checking at its first descent (unsorted ids: the first pairs)
      const int64_t up0 = from_lane_above(v[0]), up2 = from_lane_above(v[2]);
      dsc |= pair_descends(n, p0, v[0], v[1], up0, e0, lo);
      if (p0 + stride < np) dsc |= pair_descends(n, p0 + stride, v[2], v[3], up2, e2, lo);
      found = __any(dsc);
    }
    // every writer stores the same value; a read first keeps the repeats of
    // a hot id (an item rated ~5000 times) from hammering its line with stores
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (v[u] >= 0 && v[u] < span && present[v[u]] == 0) present[v[u]] = 1;
  }
  if (desc && __ballot(dsc) && (threadIdx.x & 63) == 0) atomicOr(desc, 1);
}

__global__ __launch_bounds__(256) void codes_from_rank_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t lo,
                                                              int64_t span, const int32_t* __restrict__ incl,
                                                              int32_t* __restrict__ codes,
                                                              const int32_t* __restrict__ desc,
                                                              int64_t* __restrict__ starts) {
  const bool vec = ((uintptr_t)ids & 15) == 0, vst = ((uintptr_t)codes & 7) == 0;
  const bool st = starts != nullptr && *desc == 0;  // the marking pass found the ids in order
  const int64_t stride = (int64_t)gridDim.x * blockDim.x, np = (n + 1) / 2;
  auto code = [&](int64_t v) -> int32_t {  // out-of-range ids (a caller error) -> -1
    return (v >= 0 && v < span) ? incl[v] - 1 : -1;
  };
  for (int64_t p0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p0 < np; p0 += 2 * stride) {
    int64_t v[4];
    load_id_pair(ids, n, p0, lo, vec, v[0], v[1]);
    if (p0 + stride < np) {
      load_id_pair(ids, n, p0 + stride, lo, vec, v[2], v[3]);
    } else {
      v[2] = v[3] = -1;
    }
    int32_t c[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) c[u] = code(v[u]);
    if (st) {  // the code before each pair: the lane below's, or on lane 0 a scalar lookup
      const int64_t q0 = wave_prev_pos(p0), q2 = wave_prev_pos(p0 + stride);
      const int32_t e0 = q0 >= 0 && q0 < n ? code(ids[q0] - lo) : -1;
      const int32_t e2 = q2 >= 0 && q2 < n ? code(ids[q2] - lo) : -1;
      int32_t b0 = from_lane_below(c[1]), b2 = from_lane_below(c[3]);
      if ((threadIdx.x & 63) == 0) b0 = e0, b2 = e2;
      pair_starts(n, p0, c[0], c[1], b0, starts);
      if (p0 + stride < np) pair_starts(n, p0 + stride, c[2], c[3], b2, starts);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t p = p0 + h * stride;
      if (p >= np) break;
      const int32_t c0 = c[2 * h], c1 = c[2 * h + 1];
      if (vst && 2 * p + 1 < n) {
        *reinterpret_cast<int2*>(codes + 2 * p) = make_int2(c0, c1);
      } else {
        codes[2 * p] = c0;
        if (2 * p + 1 < n) codes[2 * p + 1] = c1;
      }
    }
  }
}

__global__ __launch_bounds__(256) void uniq_from_rank_kernel(const int32_t* __restrict__ present,
                                                             const int32_t* __restrict__ incl, int64_t span,
                                                             int64_t lo, int64_t* __restrict__ uniq,
                                                             int64_t* __restrict__ n_uniq) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < span; v += (int64_t)gridDim.x * blockDim.x) {
    if (present[v]) uniq[incl[v] - 1] = v + lo;
    if (v == span - 1) *n_uniq = (int64_t)incl[v];
  }
}

// Small dense spans (<= kBitsSpan ids, e.g. c2's 100k items): presence as a
// bitmap that every block keeps in LDS, ranks from per-word prefix counts —
// the random per-entry table accesses stay in LDS instead of L2 lines.
constexpr int64_t kBitsSpan = (int64_t)1 << 19;  // bitmap 64 KB + prefixes 64 KB
constexpr unsigned kBitsBlocks = 1024;

__global__ __launch_bounds__(256) void mark_bits_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t lo,
                                                        int64_t span, uint32_t* __restrict__ bits,
                                                        int32_t* __restrict__ desc) {
  extern __shared__ uint32_t lb[];
  const int nw = (int)((span + 31) >> 5);
  for (int q = threadIdx.x; q < nw; q += 256) lb[q] = 0u;
  __syncthreads();
  const bool vec = ((uintptr_t)ids & 15) == 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x, np = (n + 1) / 2;
  bool dsc = false, found = false;
  for (int64_t p0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p0 < np; p0 += 2 * stride) {
    int64_t v[4];
    load_id_pair(ids, n, p0, lo, vec, v[0], v[1]);
    if (p0 + stride < np) {
      load_id_pair(ids, n, p0 + stride, lo, vec, v[2], v[3]);
    } else {
      v[2] = v[3] = -1;
    }
    const int64_t e0 = edge_id(ids, n, p0, desc && !found), e2 = edge_id(ids, n, p0 + stride, desc && !found);
    if (desc && !found) {  // a wave stops checking at its first descent (unsorted ids: the first pairs)
      const int64_t up0 = from_lane_above(v[0]), up2 = from_lane_above(v[2]);
      dsc |= pair_descends(n, p0, v[0], v[1], up0, e0, lo);
      if (p0 + stride < np) dsc |= pair_descends(n, p0 + stride, v[2], v[3], up2, e2, lo);
      found = __any(dsc);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (v[u] >= 0 && v[u] < span) atomicOr(&lb[v[u] >> 5], 1u << (v[u] & 31));
  }
  if (desc && __ballot(dsc) && (threadIdx.x & 63) == 0) atomicOr(desc, 1);
  __syncthreads();
  for (int q = threadIdx.x; q < nw; q += 256)
    if (lb[q]) atomicOr(&bits[q], lb[q]);
}

// pre[q] = ids present below word q (one block: words <= 16384); total -> *n_uniq
__global__ __launch_bounds__(1024) void bits_prefix_kernel(const uint32_t* __restrict__ bits, int nw,
                                                           uint32_t* __restrict__ pre, int64_t* __restrict__ n_uniq) {
  __shared__ uint32_t wsum[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (int q0 = 0; q0 < nw; q0 += 1024) {
    const int q = q0 + threadIdx.x;
    const uint32_t c = q < nw ? (uint32_t)__popc(bits[q]) : 0u;
    uint32_t x = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t base = carry, tot = 0;
    for (int k = 0; k < 16; ++k) {
      if (k < w) base += wsum[k];
      tot += wsum[k];
    }
    if (q < nw) pre[q] = base + x - c;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *n_uniq = (int64_t)carry;
}

__global__ __launch_bounds__(256) void codes_bits_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t lo,
                                                         int64_t span, const uint32_t* __restrict__ bits,
                                                         const uint32_t* __restrict__ pre,
                                                         int32_t* __restrict__ codes,
                                                         const int32_t* __restrict__ desc,
                                                         int64_t* __restrict__ starts) {
  extern __shared__ uint32_t lb[];
  const int nw = (int)((span + 31) >> 5);
  uint32_t* lp = lb + nw;
  for (int q = threadIdx.x; q < nw; q += 256) {
    lb[q] = bits[q];
    lp[q] = pre[q];
  }
  __syncthreads();
  const bool vec = ((uintptr_t)ids & 15) == 0, vst = ((uintptr_t)codes & 7) == 0;
  const bool st = starts != nullptr && *desc == 0;  // the marking pass found the ids in order
  const int64_t stride = (int64_t)gridDim.x * blockDim.x, np = (n + 1) / 2;
  auto code = [&](int64_t v) -> int32_t {
    if (v < 0 || v >= span) return -1;  // out of range (a caller error)
    const uint32_t wd = lb[v >> 5];
    return (int32_t)(lp[v >> 5] + (uint32_t)__popc(wd & ((1u << (v & 31)) - 1u)));
  };
  for (int64_t p0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p0 < np; p0 += 2 * stride) {
    int64_t v[4];
    load_id_pair(ids, n, p0, lo, vec, v[0], v[1]);
    if (p0 + stride < np) {
      load_id_pair(ids, n, p0 + stride, lo, vec, v[2], v[3]);
    } else {
      v[2] = v[3] = -1;
    }
    int32_t c[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) c[u] = code(v[u]);
    if (st) {  // as codes_from_rank_kernel
      const int64_t q0 = wave_prev_pos(p0), q2 = wave_prev_pos(p0 + stride);
      const int32_t e0 = q0 >= 0 && q0 < n ? code(ids[q0] - lo) : -1;
      const int32_t e2 = q2 >= 0 && q2 < n ? code(ids[q2] - lo) : -1;
      int32_t b0 = from_lane_below(c[1]), b2 = from_lane_below(c[3]);
      if ((threadIdx.x & 63) == 0) b0 = e0, b2 = e2;
      pair_starts(n, p0, c[0], c[1], b0, starts);
      if (p0 + stride < np) pair_starts(n, p0 + stride, c[2], c[3], b2, starts);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t p = p0 + h * stride;
      if (p >= np) break;
      const int32_t c0 = c[2 * h], c1 = c[2 * h + 1];
      if (vst && 2 * p + 1 < n) {
        *reinterpret_cast<int2*>(codes + 2 * p) = make_int2(c0, c1);
      } else {
        codes[2 * p] = c0;
        if (2 * p + 1 < n) codes[2 * p + 1] = c1;
      }
    }
  }
}

__global__ __launch_bounds__(256) void uniq_bits_kernel(const uint32_t* __restrict__ bits,
                                                        const uint32_t* __restrict__ pre, int64_t span, int64_t lo,
                                                        int64_t* __restrict__ uniq) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < span; v += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t wd = bits[v >> 5];
    if ((wd >> (v & 31)) & 1u) uniq[pre[v >> 5] + (uint32_t)__popc(wd & ((1u << (v & 31)) - 1u))] = v + lo;
  }
}

// Row starts of the codes (the sorting paths of hrec_encode_ids_ex; skipped
// unless the ids were found in order): as pair_starts, one position a thread.
__global__ __launch_bounds__(256) void code_starts_kernel(const int32_t* __restrict__ codes, int64_t n,
                                                          const int32_t* __restrict__ desc,
                                                          int64_t* __restrict__ starts) {
  if (*desc != 0) return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t c = codes[i];
    if (c < 0) continue;
    if (i == 0 || codes[i - 1] != c) starts[c] = i;
    if (i == n - 1) starts[c + 1] = n;
  }
}

// indptr from row-sorted keys: indptr[r] = first i with keys[i] >= r.
// Each boundary between distinct keys fills the empty rows in between.
__global__ __launch_bounds__(256) void indptr_from_sorted_kernel(const int32_t* __restrict__ keys, int64_t nnz,
                                                                 int64_t n_rows, int64_t* __restrict__ indptr) {
  // thread j: positions 4j .. 4j + 3 (one 16-B load when aligned and in range)
  const bool vec = ((uintptr_t)keys & 15) == 0;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; 4 * j <= nnz;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = 4 * j;
    int64_t k[4];
    if (vec && i0 + 3 < nnz) {
      const int4 v = *reinterpret_cast<const int4*>(keys + i0);
      k[0] = v.x, k[1] = v.y, k[2] = v.z, k[3] = v.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) k[e] = i0 + e < nnz ? (int64_t)keys[i0 + e] : n_rows;
    }
    int64_t lo = i0 == 0 ? -1 : (int64_t)keys[i0 - 1];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t i = i0 + e;
      if (i > nnz) break;
      const int64_t hi = i == nnz ? n_rows : k[e];
      for (int64_t r = lo + 1; r <= hi && r <= n_rows; ++r) indptr[r] = i;
      lo = hi;
    }
  }
}

// indptr[r] = min(first[r], first[r + 1], ...) from the end: rows without
// entries take the next row's start (first[] holds each present key's first
// position, nnz elsewhere; indptr[n_rows] = nnz). Tiles of kMinTile rows:
// the tiles' minima (one block each), then per tile the minimum of the tiles
// after it and a suffix min of its rows (a thread's 8 rows in registers, a
// wave / block suffix scan of the threads' minima).
constexpr int kMinThreads = 1024, kMinPer = 8, kMinTile = kMinThreads * kMinPer;

__device__ __forceinline__ unsigned long long umin64(unsigned long long a, unsigned long long b) { return a < b ? a : b; }

// block-wide min over kMinThreads values; every thread gets the result
__device__ __forceinline__ unsigned long long block_min64(unsigned long long m, unsigned long long* sh) {
  for (int off = 32; off >= 1; off >>= 1) m = umin64(m, __shfl_xor(m, off, 64));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = m;
  __syncthreads();
  m = ~0ull;
  for (int q = 0; q < kMinThreads / 64; ++q) m = umin64(m, sh[q]);
  return m;
}

__global__ __launch_bounds__(kMinThreads) void indptr_tile_min_kernel(const unsigned long long* __restrict__ first,
                                                                      int64_t n, unsigned long long* __restrict__ tmin) {
  __shared__ unsigned long long sh[kMinThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kMinTile;
  unsigned long long m = ~0ull;
#pragma unroll
  for (int e = 0; e < kMinPer; ++e) {
    const int64_t r = base + (int64_t)e * kMinThreads + threadIdx.x;
    if (r < n) m = umin64(m, first[r]);
  }
  m = block_min64(m, sh);
  if (threadIdx.x == 0) tmin[blockIdx.x] = m;
}

__global__ __launch_bounds__(kMinThreads) void indptr_suffix_min_kernel(unsigned long long* __restrict__ first,
                                                                        int64_t n,
                                                                        const unsigned long long* __restrict__ tmin,
                                                                        int64_t n_tiles) {
  __shared__ unsigned long long sh[kMinThreads / 64];
  // the tiles after this one
  unsigned long long carry = ~0ull;
  for (int64_t t = blockIdx.x + 1 + threadIdx.x; t < n_tiles; t += kMinThreads) carry = umin64(carry, tmin[t]);
  carry = block_min64(carry, sh);
  // thread t: rows base + 8t .. 8t + 7
  const int64_t r0 = (int64_t)blockIdx.x * kMinTile + (int64_t)threadIdx.x * kMinPer;
  unsigned long long v[kMinPer];
#pragma unroll
  for (int e = 0; e < kMinPer; ++e) v[e] = r0 + e < n ? first[r0 + e] : ~0ull;
#pragma unroll
  for (int e = kMinPer - 2; e >= 0; --e) v[e] = umin64(v[e], v[e + 1]);
  // suffix min over the threads above (lanes, then waves)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned long long x = v[0];
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long y = __shfl_down(x, off, 64);
    if (lane + off < 64) x = umin64(x, y);
  }
  __syncthreads();
  if (lane == 0) sh[w] = x;  // the wave's minimum
  __syncthreads();
  unsigned long long after = carry;
  for (int q = w + 1; q < kMinThreads / 64; ++q) after = umin64(after, sh[q]);
  const unsigned long long up = __shfl_down(x, 1, 64);  // the lanes above within the wave
  if (lane < 63) after = umin64(after, up);
#pragma unroll
  for (int e = 0; e < kMinPer; ++e)
    if (r0 + e < n) first[r0 + e] = umin64(v[e], after);
}

__global__ __launch_bounds__(256) void fill_u64_kernel(unsigned long long* __restrict__ x, int64_t n,
                                                       unsigned long long v) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) x[i] = v;
}

// ---------------------------------------------------------------- CSR build
// Stable LSD radix sort of the row codes carrying (col, rating), written for
// this shape: dense codes < n_rows, so ceil(bits / 10) passes of <= 10-bit
// digits (c2's CSC: 100k item codes = 17 bits = 2 passes of 8 + 9 bits, the
// wider digit last). Per pass:
//   1. upsweep: per tile of kSortTile entries, the digit histogram (LDS
//      atomics) -> counts[tile][digit];
//   2. a column scan of the tile-major counts (sort_colsum / colscan_*): the
//      output offset of every (tile, digit) — digits ascending, tiles in
//      input order;
//   3. downsweep (persistent, one block per CU; the next tile's entries load
//      while a tile is written out): each wave takes a contiguous 1/8 of the
//      block's tile into registers and ranks its entries among its own same-digit entries in
//      input order (per 64-entry round: the lanes below with the same digit,
//      from `bits` ballots, plus the wave's running per-digit count in LDS —
//      no block barriers); one scan over (digit, wave) turns the per-wave
//      counts into offsets in the tile's digit-sorted order; the tile is
//      sorted in LDS and written out, so each digit's entries leave as one
//      coalesced run at the (digit, tile) offset: a stable scatter with
//      per-block ranks. The last pass writes indices / values unpacked; the
//      first reads cols / values unpacked.
#ifndef HREC_SORT_IPT
#define HREC_SORT_IPT 20
#endif
#ifndef HREC_SORT_BPC
#define HREC_SORT_BPC 1
#endif
#ifndef HREC_SORT_NT
#define HREC_SORT_NT 0
#endif
#ifndef HREC_SORT_NTL
#define HREC_SORT_NTL 0
#endif
template <typename T>
__device__ __forceinline__ void sort_st(T* p, T v) {
  if constexpr (HREC_SORT_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <typename T>
__device__ __forceinline__ T sort_ld(const T* p) {
  if constexpr (HREC_SORT_NTL) return __builtin_nontemporal_load(p);
  else return *p;
}
constexpr int kSortThreads = 512, kSortIPT = HREC_SORT_IPT, kSortTile = kSortThreads * kSortIPT;  // 10240 entries
constexpr int kSortMaxBits = 10;
static_assert(kSortIPT % 4 == 0, "the upsweep's 16-B key loads");

// Persistent blocks (4 per CU) walk the tiles; the next tile's keys are
// loaded (16-B loads where aligned) before this tile's LDS histogram.
constexpr int kUpBlocksPerCU = 4;

__global__ __launch_bounds__(kSortThreads) void sort_upsweep_kernel(const int32_t* __restrict__ keys, int64_t n,
                                                                    int shift, int bits, int64_t n_tiles,
                                                                    uint32_t* __restrict__ counts) {
  __shared__ uint32_t h[1 << kSortMaxBits];
  constexpr int NV = kSortIPT / 4;  // 16-B loads per thread and tile
  const int R = 1 << bits;
  const uint32_t dmask = (uint32_t)(R - 1);
  const bool vec = ((uintptr_t)keys & 15) == 0;
  int4 cur[NV], nxt[NV];
  auto load = [&](int64_t tile, int4* k) {
    const int64_t base = tile * kSortTile;
    if (tile >= n_tiles) return;
    if (vec && base + kSortTile <= n) {
#pragma unroll
      for (int e = 0; e < NV; ++e)
        k[e] = *reinterpret_cast<const int4*>(keys + base + 4 * ((int64_t)e * kSortThreads + threadIdx.x));
    } else {
#pragma unroll
      for (int e = 0; e < NV; ++e) {
        const int64_t i = base + 4 * ((int64_t)e * kSortThreads + threadIdx.x);
        k[e].x = i < n ? keys[i] : -1;
        k[e].y = i + 1 < n ? keys[i + 1] : -1;
        k[e].z = i + 2 < n ? keys[i + 2] : -1;
        k[e].w = i + 3 < n ? keys[i + 3] : -1;
      }
    }
  };
  int64_t tile = blockIdx.x;
  load(tile, cur);
  for (; tile < n_tiles; tile += gridDim.x) {
    load(tile + gridDim.x, nxt);
    for (int d = threadIdx.x; d < R; d += kSortThreads) h[d] = 0;
    __syncthreads();
    const int64_t base = tile * kSortTile;
    const bool full = base + kSortTile <= n;
#pragma unroll
    for (int e = 0; e < NV; ++e) {
      const int64_t i = base + 4 * ((int64_t)e * kSortThreads + threadIdx.x);
      const int32_t kv[4] = {cur[e].x, cur[e].y, cur[e].z, cur[e].w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (full || i + q < n) atomicAdd(&h[((uint32_t)kv[q] >> shift) & dmask], 1u);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < R; d += kSortThreads) counts[tile * R + d] = h[d];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < NV; ++e) cur[e] = nxt[e];
  }
}

// counts [tile][digit] (tile-major: every access below reads or writes whole
// rows) -> in place, the output offset of (tile, digit) = the entries of all
// smaller digits + the entries of this digit in earlier tiles. Column sums
// per chunk of kScanTiles tiles, one block scans them (per digit over the
// chunks, then the digit totals), chunks add their running prefix.
constexpr int kScanTiles = 256;

__global__ __launch_bounds__(512) void sort_colsum_kernel(const uint32_t* __restrict__ cnt, int64_t n_tiles, int R,
                                                          uint32_t* __restrict__ csum) {
  const int64_t t0 = (int64_t)blockIdx.x * kScanTiles;
  const int64_t t1 = t0 + kScanTiles < n_tiles ? t0 + kScanTiles : n_tiles;
  for (int d = threadIdx.x; d < R; d += 512) {
    uint32_t a = 0;
#pragma unroll 8
    for (int64_t t = t0; t < t1; ++t) a += cnt[t * R + d];
    csum[(int64_t)blockIdx.x * R + d] = a;
  }
}

__global__ __launch_bounds__(1024) void sort_colscan_top_kernel(uint32_t* __restrict__ csum, int64_t n_chunks, int R) {
  __shared__ uint32_t tot[1 << kSortMaxBits];
  __shared__ uint32_t wsum[16];
  const int d = threadIdx.x;  // R <= 1024 = blockDim
  uint32_t run = 0;
  if (d < R)  // 8 loads in flight per step (not one dependent load per chunk)
    for (int64_t c0 = 0; c0 < n_chunks; c0 += 8) {
      uint32_t v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = c0 + j < n_chunks ? csum[(c0 + j) * R + d] : 0u;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (c0 + j < n_chunks) {
          csum[(c0 + j) * R + d] = run;
          run += v[j];
        }
    }
  // exclusive scan of the digit totals
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = d < R ? run : 0;
  const uint32_t mine = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t base = x - mine;
  for (int q = 0; q < w; ++q) base += wsum[q];
  tot[d] = base;
  __syncthreads();
  if (d < R) {
    const uint32_t t = tot[d];
    for (int64_t c0 = 0; c0 < n_chunks; c0 += 8) {
      uint32_t v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = c0 + j < n_chunks ? csum[(c0 + j) * R + d] : 0u;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (c0 + j < n_chunks) csum[(c0 + j) * R + d] = v[j] + t;
    }
  }
}

__global__ __launch_bounds__(512) void sort_colscan_apply_kernel(uint32_t* __restrict__ cnt, int64_t n_tiles, int R,
                                                                 const uint32_t* __restrict__ csum) {
  const int64_t t0 = (int64_t)blockIdx.x * kScanTiles;
  const int64_t t1 = t0 + kScanTiles < n_tiles ? t0 + kScanTiles : n_tiles;
  for (int d = threadIdx.x; d < R; d += 512) {
    uint32_t run = csum[(int64_t)blockIdx.x * R + d];
    for (int64_t tb = t0; tb < t1; tb += 8) {
      uint32_t v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = tb + j < t1 ? cnt[(tb + j) * R + d] : 0u;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (tb + j < t1) {
          cnt[(tb + j) * R + d] = run;
          run += v[j];
        }
    }
  }
}

// LAST with imin != nullptr (the CSR build): the sorted keys are not written;
// each key's first position goes to imin[key] by atomicMin (the first entry of
// every distinct key of a tile's digit run — runs are sorted by the whole key,
// earlier passes sorted the low digits), and indptr_suffix_min_kernel fills
// the empty rows: no keys written, no indptr pass re-reading them.
template <bool FIRST, bool LAST>
__global__ __launch_bounds__(kSortThreads) void sort_downsweep_kernel(
    const int32_t* __restrict__ keys_in, const int32_t* __restrict__ cols_in, const float* __restrict__ vals_in,
    const uint64_t* __restrict__ pay_in, int64_t n, int shift, int bits, int64_t n_tiles,
    const uint32_t* __restrict__ offs, int32_t* __restrict__ keys_out, uint64_t* __restrict__ pay_out,
    int32_t* __restrict__ idx_out, float* __restrict__ val_out, unsigned long long* __restrict__ imin,
    int64_t imin_n) {
  constexpr int R_MAX = 1 << kSortMaxBits, NW = kSortThreads / 64, PW = kSortTile / NW;  // entries per wave
  __shared__ int32_t sk[kSortTile];                 // the tile, sorted by digit (stable)
  __shared__ uint64_t sp[kSortTile];
  __shared__ uint16_t wh[NW][R_MAX];                // per wave and digit: count, then the wave's tile offset
  __shared__ uint32_t goff[R_MAX];                  // per digit: the tile's first output position
  __shared__ uint32_t scan_sh[NW];
  const int R = 1 << bits;
  const uint32_t dmask = (uint32_t)(R - 1);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  // wave w takes tile entries [w PW, (w + 1) PW), 64 per round (coalesced)
  int32_t key[kSortIPT];
  uint64_t pay[kSortIPT];
  auto load = [&](int64_t tile) {
    const int64_t base = tile * kSortTile;
#pragma unroll
    for (int r = 0; r < kSortIPT; ++r) {
      const int64_t i = base + w * PW + r * 64 + lane;
      key[r] = 0;
      pay[r] = 0;
      if (tile < n_tiles && i < n) {
        key[r] = sort_ld(keys_in + i);
        if constexpr (FIRST) {
          pay[r] = (uint64_t)(uint32_t)sort_ld(cols_in + i) | ((uint64_t)__float_as_uint(sort_ld(vals_in + i)) << 32);
        } else {
          pay[r] = sort_ld(pay_in + i);
        }
      }
    }
  };
  // persistent blocks (one per CU: the tile takes 118 KB of LDS); the next
  // tile's entries and digit offsets load while this tile is written out
  uint32_t go[2];  // offsets of digits t, t + 512 (R <= 1024)
  auto load_offs = [&](int64_t tile) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int d = threadIdx.x + h * kSortThreads;
      go[h] = (tile < n_tiles && d < R) ? offs[tile * R + d] : 0u;
    }
  };
  int64_t tile = blockIdx.x;
  load(tile);
  load_offs(tile);
  for (; tile < n_tiles; tile += gridDim.x) {
    const int64_t base = tile * kSortTile;
    const int tn = (int)(n - base < kSortTile ? n - base : kSortTile);  // entries of this tile
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int d = threadIdx.x + h * kSortThreads;
      if (d < R) {
        goff[d] = go[h];
#pragma unroll
        for (int q = 0; q < NW; ++q) wh[q][d] = 0;
      }
    }
    __syncthreads();
    // 1. each wave ranks its own entries in order (no block barriers): within
    //    a round the lanes below with the same digit (peer mask from `bits`
    //    ballots), before it the wave's running per-digit count (LDS)
    uint32_t rk[kSortIPT];
#pragma unroll
    for (int r = 0; r < kSortIPT; ++r) {
      const bool active = w * PW + r * 64 + lane < tn;
      const uint32_t dg = ((uint32_t)key[r] >> shift) & dmask;
      uint64_t peers = __ballot(active);
      for (int b = 0; b < bits; ++b) {
        const uint64_t m = __ballot((dg >> b) & 1u);
        peers &= ((dg >> b) & 1u) ? m : ~m;
      }
      const int rank = __popcll(peers & lt);
      const uint32_t before = active ? wh[w][dg] : 0;
      rk[r] = before + (uint32_t)rank;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (active && rank == 0) wh[w][dg] = (uint16_t)(before + __popcll(peers));
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __syncthreads();
    // 2. offsets in the tile's digit-sorted order: digits ascending, waves in
    //    order within a digit (exclusive scan over (digit, wave); thread t
    //    owns digits 2t, 2t + 1, R <= 1024)
    {
      const int d0 = 2 * threadIdx.x;
      uint32_t c[2][NW], tot = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          c[h][q] = d0 + h < R ? wh[q][d0 + h] : 0;
          tot += c[h][q];
        }
      uint32_t x = tot;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
      }
      if (lane == 63) scan_sh[w] = x;
      __syncthreads();
      uint32_t run = x - tot;
      for (int q = 0; q < w; ++q) run += scan_sh[q];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          if (d0 + h < R) wh[q][d0 + h] = (uint16_t)run;
          run += c[h][q];
        }
    }
    __syncthreads();
    // 3. the tile sorted into LDS; then the next tile's loads are issued
#pragma unroll
    for (int r = 0; r < kSortIPT; ++r) {
      if (w * PW + r * 64 + lane < tn) {
        const uint32_t dg = ((uint32_t)key[r] >> shift) & dmask;
        const uint32_t q = wh[w][dg] + rk[r];
        sk[q] = key[r];
        sp[q] = pay[r];
      }
    }
    __syncthreads();
    load(tile + gridDim.x);
    load_offs(tile + gridDim.x);
    // 4. write out: consecutive LDS entries of one digit go to consecutive
    //    output positions (coalesced runs); a digit's first LDS slot is its
    //    wave-0 offset
#pragma unroll
    for (int e = 0; e < kSortIPT; ++e) {
      const int q = e * kSortThreads + threadIdx.x;
      if (q >= tn) break;
      const int32_t k = sk[q];
      const uint32_t dg = ((uint32_t)k >> shift) & dmask;
      const uint32_t pos = goff[dg] + ((uint32_t)q - wh[0][dg]);
      const uint64_t pv = sp[q];
      if (!LAST || imin == nullptr) {
        sort_st(keys_out + pos, k);
      } else if (((uint32_t)q == wh[0][dg] || sk[q - 1] != k) && (uint32_t)k < (uint64_t)imin_n) {
        atomicMin(&imin[(uint32_t)k], (unsigned long long)pos);  // the run's first entry of key k
      }
      if constexpr (LAST) {
        sort_st(idx_out + pos, (int32_t)(uint32_t)pv);
        sort_st(val_out + pos, __uint_as_float((uint32_t)(pv >> 32)));
      } else {
        sort_st(pay_out + pos, pv);
      }
    }
    __syncthreads();
  }
}

// *flag = 1 if some x[i] > x[i + 1] (the caller zeroes it first)
template <typename T>
__global__ __launch_bounds__(256) void descent_kernel(const T* __restrict__ x, int64_t n, int32_t* __restrict__ flag) {
  bool d = false;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 + 1 < n; i0 += kStreamUnroll * stride) {
#pragma unroll
    for (int u = 0; u < kStreamUnroll; ++u) {
      const int64_t i = i0 + u * stride;
      if (i + 1 < n) d |= x[i] > x[i + 1];
    }
    // stop once any wave has found a descent (unsorted input: the common
    // case for the CSC rows ends after the grid's first pass)
    if (__any(d)) {
      if ((threadIdx.x & 63) == 0) *flag = 1;
      return;
    }
    if (*reinterpret_cast<volatile const int32_t*>(flag)) return;
  }
}

// rows already non-decreasing: the CSR is the input order (the stable sort is the identity)
__global__ __launch_bounds__(256) void copy_entries_kernel(const int32_t* __restrict__ cols, const float* __restrict__ vals,
                                                           int64_t nnz, int32_t* __restrict__ indices,
                                                           float* __restrict__ values) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < nnz; i0 += kStreamUnroll * stride) {
    int32_t c[kStreamUnroll];
    float v[kStreamUnroll];
#pragma unroll
    for (int u = 0; u < kStreamUnroll; ++u)
      if (i0 + u * stride < nnz) {
        c[u] = cols[i0 + u * stride];
        v[u] = vals[i0 + u * stride];
      }
#pragma unroll
    for (int u = 0; u < kStreamUnroll; ++u)
      if (i0 + u * stride < nnz) {
        indices[i0 + u * stride] = c[u];
        values[i0 + u * stride] = v[u];
      }
  }
}

inline unsigned grid_for(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < 65536 ? (b > 0 ? b : 1) : 65536);
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

int bits_for(int64_t n_rows) {  // radix bits covering codes 0 .. n_rows-1
  int b = 1;
  while (b < 32 && ((int64_t)1 << b) < n_rows) ++b;
  return b;
}

// CSR build workspace: ping-pong keys / packed (col, rating) entries of the
// intermediate passes, the (digit, tile) counts and the scan's chunk sums.
struct CsrWs {
  size_t ka, kb, pa, pb, cnt, sums, total;
  int passes, digit[4];
  int64_t n_tiles, n_cnt, n_chunks;
  CsrWs(int64_t nnz, int bits) {
    passes = (bits + kSortMaxBits - 1) / kSortMaxBits;
    if (passes < 1) passes = 1;
#ifndef HREC_SORT_WIDE_LAST
#define HREC_SORT_WIDE_LAST 1
#endif
    // the wider digits first (HREC_SORT_WIDE_LAST=1: last)
    for (int p = 0; p < passes; ++p)
      digit[p] = bits / passes + ((HREC_SORT_WIDE_LAST ? p >= passes - bits % passes : p < bits % passes) ? 1 : 0);
    n_tiles = (nnz + kSortTile - 1) / kSortTile;
    int maxd = 0;
    for (int p = 0; p < passes; ++p) maxd = digit[p] > maxd ? digit[p] : maxd;
    n_cnt = ((int64_t)1 << maxd) * n_tiles;
    n_chunks = ((n_tiles + kScanTiles - 1) / kScanTiles) << maxd;  // column sums
    ka = 0;
    kb = ka + align256(4 * (size_t)nnz);
    pa = kb + align256(4 * (size_t)nnz);
    pb = pa + align256(8 * (size_t)nnz);
    cnt = pb + align256(8 * (size_t)nnz);
    sums = cnt + align256(4 * (size_t)n_cnt);
    total = sums + align256(4 * (size_t)n_chunks);
  }
};

// The largest CsrWs over every key width (1 .. 32 bits).
inline size_t csr_ws_max(int64_t n) {
  size_t m = 0;
  for (int b = 1; b <= 32; ++b) {
    const size_t t = CsrWs(n, b).total;
    m = t > m ? t : m;
  }
  return m;
}

// Workspace layout of hrec_encode_ids (all 256-B aligned): the shifted
// 32-bit keys (or, for id spans past 2^32, the sorted 64-bit keys), the
// position columns, the distinct flags and their scan, and a temp region for
// the in-tree radix sort (its workspace, then four 32-bit columns for the
// two-word sort of spans past 2^32) or the scan.
struct EncodeWs {
  size_t keys, pos, pos2, flag, incl, temp, total;
  explicit EncodeWs(int64_t n) {
    // the in-tree sort's workspace (its sorted keys stay there), the sort's
    // value output, then the scan's workspace (must not overlap the keys)
    size_t tmp = csr_ws_max(n) + align256(4 * (size_t)n) + align256(scan_ws_bytes(n));
    const size_t wide = csr_ws_max(n) + 4 * align256(4 * (size_t)n);
    if (wide > tmp) tmp = wide;
    if (scan_ws_bytes(n) > tmp) tmp = scan_ws_bytes(n);
    keys = 0;
    pos = keys + align256(8 * (size_t)n);
    pos2 = pos + align256(4 * (size_t)n);
    flag = pos2 + align256(4 * (size_t)n);
    incl = flag + align256(4 * (size_t)n);
    temp = incl + align256(4 * (size_t)n);
    total = temp + align256(tmp);
  }
};

// Stable sort of (key, col, val) by the low `bits` bits of the unsigned
// keys: ceil(bits / 10) LSD passes. idx_out / val_out get the cols / vals in
// key order; *sorted_keys points at the sorted keys (inside ws).
int csr_sort_run(const int32_t* keys, const int32_t* cols, const float* vals, int64_t nnz, int bits, void* ws,
                 int32_t* idx_out, float* val_out, const int32_t** sorted_keys, hipStream_t s,
                 unsigned long long* imin = nullptr, int64_t imin_n = 0) {
  const CsrWs L(nnz, bits);
  char* w = static_cast<char*>(ws);
  int32_t* kbuf[2] = {reinterpret_cast<int32_t*>(w + L.ka), reinterpret_cast<int32_t*>(w + L.kb)};
  uint64_t* pbuf[2] = {reinterpret_cast<uint64_t*>(w + L.pa), reinterpret_cast<uint64_t*>(w + L.pb)};
  uint32_t* cnt = reinterpret_cast<uint32_t*>(w + L.cnt);
  uint32_t* sums = reinterpret_cast<uint32_t*>(w + L.sums);
  // downsweep: persistent, one block per CU (its tile takes 118 KB of LDS)
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t nd_max = (int64_t)HREC_SORT_BPC * cus;
  const unsigned nd = (unsigned)(L.n_tiles < nd_max ? L.n_tiles : nd_max);
  const int32_t* kin = keys;
  const uint64_t* pin = nullptr;
  int shift = 0;
  for (int p = 0; p < L.passes; ++p) {
    const int db = L.digit[p];
    const int R = 1 << db;
    const int64_t n_chunks = (L.n_tiles + kScanTiles - 1) / kScanTiles;
    const int64_t nu_max = (int64_t)kUpBlocksPerCU * cus;
    hipLaunchKernelGGL(sort_upsweep_kernel, dim3((unsigned)(L.n_tiles < nu_max ? L.n_tiles : nu_max)),
                       dim3(kSortThreads), 0, s, kin, nnz, shift, db, L.n_tiles, cnt);
    hipLaunchKernelGGL(sort_colsum_kernel, dim3((unsigned)n_chunks), dim3(512), 0, s, cnt, L.n_tiles, R, sums);
    hipLaunchKernelGGL(sort_colscan_top_kernel, dim3(1), dim3(1024), 0, s, sums, n_chunks, R);
    hipLaunchKernelGGL(sort_colscan_apply_kernel, dim3((unsigned)n_chunks), dim3(512), 0, s, cnt, L.n_tiles, R, sums);
    const bool first = p == 0, last = p == L.passes - 1;
    int32_t* kout = kbuf[p & 1];
    uint64_t* pout = pbuf[p & 1];
#define HREC_DOWN(F, LST)                                                                                        \
  hipLaunchKernelGGL((sort_downsweep_kernel<F, LST>), dim3(nd), dim3(kSortThreads), 0, s, kin, cols, vals, pin, nnz, \
                     shift, db, L.n_tiles, cnt, kout, pout, idx_out, val_out, imin, imin_n)
    if (first && last) HREC_DOWN(true, true);
    else if (first) HREC_DOWN(true, false);
    else if (last) HREC_DOWN(false, true);
    else HREC_DOWN(false, false);
#undef HREC_DOWN
    const int rc = check_launch("radix sort pass");
    if (rc) return rc;
    kin = kout;
    pin = pout;
    shift += db;
  }
  *sorted_keys = kin;
  return HREC_OK;
}

size_t radix_pairs_ws_bytes(int64_t n) { return csr_ws_max(n); }

int radix_pairs_sort(const uint32_t* keys, const uint32_t* p0, const uint32_t* p1, int64_t n, int bits, void* ws,
                     uint32_t* p0_out, uint32_t* p1_out, const uint32_t** keys_sorted, hipStream_t s) {
  const int32_t* ks = nullptr;
  const int rc = csr_sort_run(reinterpret_cast<const int32_t*>(keys), reinterpret_cast<const int32_t*>(p0),
                              reinterpret_cast<const float*>(p1), n, bits, ws, reinterpret_cast<int32_t*>(p0_out),
                              reinterpret_cast<float*>(p1_out), &ks, s);
  *keys_sorted = reinterpret_cast<const uint32_t*>(ks);
  return rc;
}

// ids spanning more than 2^32: (id - lo) split into 32-bit words ...
__global__ __launch_bounds__(256) void split_u64_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t lo,
                                                        uint32_t* __restrict__ w_lo, uint32_t* __restrict__ w_hi) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint64_t d = (uint64_t)ids[i] - (uint64_t)lo;
    w_lo[i] = (uint32_t)d;
    w_hi[i] = (uint32_t)(d >> 32);
  }
}
// ... and joined back after the two sorts (the sorted ids themselves)
__global__ __launch_bounds__(256) void join_u64_kernel(const uint32_t* __restrict__ w_lo,
                                                       const uint32_t* __restrict__ w_hi, int64_t n, int64_t lo,
                                                       int64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = (int64_t)((uint64_t)lo + (((uint64_t)w_hi[i] << 32) | w_lo[i]));
}

}  // namespace hrec

using namespace hrec;

extern "C" size_t hrec_encode_ids_workspace_bytes(int64_t n) {
  if (n <= 0 || n >= 0x7fffffffll) return 0;
  return EncodeWs(n).total;
}

extern "C" int hrec_encode_ids_ex(const int64_t* ids, int64_t n, int64_t id_lo, int64_t id_hi, int64_t* uniq,
                                  int64_t* n_uniq, int32_t* codes, int32_t* descending, int64_t* starts,
                                  void* ws, size_t ws_bytes, void* stream) {
  HREC_REQUIRE(n >= 0 && n < 0x7fffffffll, "encode_ids: n=%lld out of range [0, 2^31-1)", (long long)n);
  HREC_REQUIRE(n_uniq, "encode_ids: null n_uniq");
  HREC_REQUIRE(id_lo <= id_hi, "encode_ids: id_lo > id_hi");
  HREC_REQUIRE(!starts || descending, "encode_ids: starts needs the descending flag");
  hipStream_t s = as_stream(stream);
  if (descending && hipMemsetAsync(descending, 0, sizeof(int32_t), s) != hipSuccess)
    return check_launch("encode_ids: memset");
  if (n == 0) {
    if (hipMemsetAsync(n_uniq, 0, sizeof(int64_t), s) != hipSuccess) return check_launch("encode_ids: memset");
    if (starts && hipMemsetAsync(starts, 0, sizeof(int64_t), s) != hipSuccess)
      return check_launch("encode_ids: memset");
    return HREC_OK;
  }
  HREC_REQUIRE(ids && uniq && codes && ws, "encode_ids: null pointer");
  const EncodeWs L(n);
  HREC_REQUIRE(ws_bytes >= L.total, "encode_ids: workspace %zu < %zu bytes", ws_bytes, L.total);
  char* w = static_cast<char*>(ws);
  int32_t* pos = reinterpret_cast<int32_t*>(w + L.pos);
  int32_t* pos2 = reinterpret_cast<int32_t*>(w + L.pos2);
  int32_t* flag = reinterpret_cast<int32_t*>(w + L.flag);
  int32_t* incl = reinterpret_cast<int32_t*>(w + L.incl);
  void* temp = w + L.temp;
  const unsigned g = grid_for(n);
  // A narrow id range sorts (id - lo) on only the bits it spans.
  const bool narrow = (uint64_t)id_hi - (uint64_t)id_lo < 0x7fffffffull;
  const bool span32 = (uint64_t)id_hi - (uint64_t)id_lo <= 0xffffffffull;
  const int64_t span = span32 ? (int64_t)((uint64_t)id_hi - (uint64_t)id_lo) + 1 : 0;
  if (narrow && span <= n && span <= kBitsSpan) {
    // small dense range: LDS bitmaps (flag holds the bits, incl the word prefixes)
    const int nw = (int)((span + 31) >> 5);
    uint32_t* bits = reinterpret_cast<uint32_t*>(flag);
    uint32_t* pre = reinterpret_cast<uint32_t*>(incl);
    if (hipMemsetAsync(bits, 0, (size_t)nw * sizeof(uint32_t), s) != hipSuccess)
      return check_launch("encode_ids: memset");
    const unsigned gb = g < kBitsBlocks ? g : kBitsBlocks;
    hipLaunchKernelGGL(mark_bits_kernel, dim3(gb), dim3(256), (size_t)nw * 4, s, ids, n, id_lo, span, bits,
                       descending);
    hipLaunchKernelGGL(bits_prefix_kernel, dim3(1), dim3(1024), 0, s, bits, nw, pre, n_uniq);
    const auto kfn = codes_bits_kernel;
    if (!allow_max_lds(kfn)) return check_launch("encode_ids: LDS attribute");
    hipLaunchKernelGGL(kfn, dim3(gb), dim3(256), (size_t)nw * 8, s, ids, n, id_lo, span, bits, pre, codes, descending,
                       starts);
    hipLaunchKernelGGL(uniq_bits_kernel, dim3(grid_for(span)), dim3(256), 0, s, bits, pre, span, id_lo, uniq);
    return check_launch("encode_ids: dense bitmap");
  }
  if (narrow && span <= n && span < 0x7fffffffll) {
    // dense range: the span-long tables fit the flag / incl buffers (n entries each)
    if (hipMemsetAsync(flag, 0, (size_t)span * sizeof(int32_t), s) != hipSuccess)
      return check_launch("encode_ids: memset");
    hipLaunchKernelGGL(mark_present_kernel, dim3(g), dim3(256), 0, s, ids, n, id_lo, span, flag, descending);
    const int rc = scan_run<int32_t>(flag, incl, span, false, temp, s);
    if (rc) return rc;
    hipLaunchKernelGGL(codes_from_rank_kernel, dim3(g), dim3(256), 0, s, ids, n, id_lo, span, incl, codes, descending,
                       starts);
    hipLaunchKernelGGL(uniq_from_rank_kernel, dim3(grid_for(span)), dim3(256), 0, s, flag, incl, span, id_lo, uniq,
                       n_uniq);
    return check_launch("encode_ids: dense");
  }
  if (descending && n > 1)  // the sorting paths: one more pass over the ids
    hipLaunchKernelGGL(descent_kernel<int64_t>, dim3(g), dim3(256), 0, s, ids, n, descending);
  hipLaunchKernelGGL(iota_i32_kernel, dim3(g), dim3(256), 0, s, pos, n);
  if (span32) {
    // (id - lo) as 32-bit keys, sorted with their positions by the in-tree
    // stable radix sort on the bits the span needs
    int32_t* k32 = reinterpret_cast<int32_t*>(w + L.keys);
    const int bits = span > ((int64_t)1 << 31) ? 32 : bits_for(span);
    hipLaunchKernelGGL(shift_keys_kernel, dim3(g), dim3(256), 0, s, ids, n, id_lo, k32);
    float* vdummy = reinterpret_cast<float*>(static_cast<char*>(temp) + csr_ws_max(n));
    const int32_t* k32s = nullptr;
    int rc = csr_sort_run(k32, pos, reinterpret_cast<const float*>(pos), n, bits, temp, pos2, vdummy, &k32s, s);
    if (rc) return rc;
    hipLaunchKernelGGL(distinct_flags_kernel<int32_t>, dim3(g), dim3(256), 0, s, k32s, n, flag);
    // the sorted keys live at the start of temp: the scan works past them
    void* scan_ws = static_cast<char*>(temp) + csr_ws_max(n) + align256(4 * (size_t)n);
    rc = scan_run<int32_t>(flag, incl, n, false, scan_ws, s);
    if (rc) return rc;
    hipLaunchKernelGGL(scatter_codes_kernel<int32_t>, dim3(g), dim3(256), 0, s, k32s, id_lo, pos2, flag, incl, n,
                       codes, uniq, n_uniq);
  } else {
    // ids spanning more than 2^32 (only through the C-ABI: the drop-in API's
    // ids are Spark Ints): (id - lo) as two 32-bit words, the in-tree stable
    // sort by the low word carrying (high word, position), then by the high
    // word carrying (low word, position) — LSD over 64 bits
    char* t4 = static_cast<char*>(temp) + csr_ws_max(n);
    const size_t c4 = align256(4 * (size_t)n);
    uint32_t* A = reinterpret_cast<uint32_t*>(t4);
    uint32_t* Bw = reinterpret_cast<uint32_t*>(t4 + c4);
    uint32_t* C = reinterpret_cast<uint32_t*>(t4 + 2 * c4);
    uint32_t* D = reinterpret_cast<uint32_t*>(t4 + 3 * c4);
    hipLaunchKernelGGL(split_u64_kernel, dim3(g), dim3(256), 0, s, ids, n, id_lo, A, Bw);
    const uint32_t* ks = nullptr;
    int rc = radix_pairs_sort(A, Bw, reinterpret_cast<const uint32_t*>(pos), n, 32, temp, C,
                              reinterpret_cast<uint32_t*>(pos2), &ks, s);  // C: high words, pos2: positions
    if (rc) return rc;
    if (hipMemcpyAsync(D, ks, 4 * (size_t)n, hipMemcpyDeviceToDevice, s) != hipSuccess)  // the low words, sorted
      return check_launch("encode_ids: copy");
    const uint64_t hi_span = ((uint64_t)id_hi - (uint64_t)id_lo) >> 32;
    rc = radix_pairs_sort(C, D, reinterpret_cast<const uint32_t*>(pos2), n, bits_for((int64_t)hi_span + 1), temp, A,
                          reinterpret_cast<uint32_t*>(pos), &ks, s);  // A: low words, pos: positions
    if (rc) return rc;
    int64_t* keys = reinterpret_cast<int64_t*>(w + L.keys);
    hipLaunchKernelGGL(join_u64_kernel, dim3(g), dim3(256), 0, s, A, ks, n, id_lo, keys);
    pos2 = pos;
    hipLaunchKernelGGL(distinct_flags_kernel<int64_t>, dim3(g), dim3(256), 0, s, keys, n, flag);
    rc = scan_run<int32_t>(flag, incl, n, false, temp, s);
    if (rc) return rc;
    hipLaunchKernelGGL(scatter_codes_kernel<int64_t>, dim3(g), dim3(256), 0, s, keys, (int64_t)0, pos2, flag, incl,
                       n, codes, uniq, n_uniq);
  }
  if (starts) hipLaunchKernelGGL(code_starts_kernel, dim3(g), dim3(256), 0, s, codes, n, descending, starts);
  return check_launch("encode_ids");
}

extern "C" int hrec_encode_ids(const int64_t* ids, int64_t n, int64_t id_lo, int64_t id_hi, int64_t* uniq,
                               int64_t* n_uniq, int32_t* codes, void* ws, size_t ws_bytes, void* stream) {
  return hrec_encode_ids_ex(ids, n, id_lo, id_hi, uniq, n_uniq, codes, nullptr, nullptr, ws, ws_bytes, stream);
}

extern "C" size_t hrec_minmax_i64_workspace_bytes(int64_t n) { return n > 0 ? 256 : 0; }

extern "C" int hrec_minmax_i64(const int64_t* x, int64_t n, int64_t* out, void* ws, size_t ws_bytes,
                               void* stream) {
  HREC_REQUIRE(n > 0, "minmax_i64: n=%lld must be >= 1", (long long)n);
  HREC_REQUIRE(x && out, "minmax_i64: null pointer");
  (void)ws;
  (void)ws_bytes;  // no workspace needed (kept in the signature: ABI)
  return minmax_i64_run(x, n, out, as_stream(stream));
}

extern "C" size_t hrec_coo_to_csr_workspace_bytes(int64_t nnz, int64_t n_rows) {
  if (nnz <= 0 || nnz >= 0x7fffffffll || n_rows <= 0 || n_rows >= 0x7fffffffll) return 0;
  return CsrWs(nnz, bits_for(n_rows)).total + align256(8 * (size_t)((n_rows + 1 + kMinTile - 1) / kMinTile));
}

extern "C" int hrec_coo_to_csr(const int32_t* rows, const int32_t* cols, const float* vals, int64_t nnz,
                               int64_t n_rows, int64_t* indptr, int32_t* indices, float* values, void* ws,
                               size_t ws_bytes, void* stream) {
  HREC_REQUIRE(nnz >= 0 && nnz < 0x7fffffffll, "coo_to_csr: nnz=%lld out of range", (long long)nnz);
  HREC_REQUIRE(n_rows >= 0 && n_rows < 0x7fffffffll, "coo_to_csr: n_rows=%lld out of range", (long long)n_rows);
  HREC_REQUIRE(indptr, "coo_to_csr: null indptr");
  hipStream_t s = as_stream(stream);
  if (nnz == 0) {
    if (hipMemsetAsync(indptr, 0, sizeof(int64_t) * (size_t)(n_rows + 1), s) != hipSuccess)
      return check_launch("coo_to_csr: memset");
    return HREC_OK;
  }
  HREC_REQUIRE(n_rows > 0, "coo_to_csr: entries but no rows");
  HREC_REQUIRE(rows && cols && vals && indices && values && ws, "coo_to_csr: null pointer");
  const int bits = bits_for(n_rows);
  const CsrWs L(nnz, bits);
  const size_t need = hrec_coo_to_csr_workspace_bytes(nnz, n_rows);
  HREC_REQUIRE(ws_bytes >= need, "coo_to_csr: workspace %zu < %zu bytes", ws_bytes, need);
  // indptr: every row's first position (atomicMin in the last pass, nnz for
  // rows without entries), then a suffix min fills the empty rows
  unsigned long long* first = reinterpret_cast<unsigned long long*>(indptr);
  hipLaunchKernelGGL(fill_u64_kernel, dim3(grid_for(n_rows + 1)), dim3(256), 0, s, first, n_rows + 1,
                     (unsigned long long)nnz);
  const int32_t* kin = nullptr;
  int rc = csr_sort_run(rows, cols, vals, nnz, bits, ws, indices, values, &kin, s, first, n_rows);
  if (rc) return rc;
  const int64_t n_min_tiles = (n_rows + 1 + kMinTile - 1) / kMinTile;
  unsigned long long* tmin = reinterpret_cast<unsigned long long*>(static_cast<char*>(ws) + L.total);
  hipLaunchKernelGGL(indptr_tile_min_kernel, dim3((unsigned)n_min_tiles), dim3(kMinThreads), 0, s, first, n_rows + 1,
                     tmin);
  hipLaunchKernelGGL(indptr_suffix_min_kernel, dim3((unsigned)n_min_tiles), dim3(kMinThreads), 0, s, first,
                     n_rows + 1, tmin, n_min_tiles);
  return check_launch("coo_to_csr");
}

extern "C" int hrec_rows_descending_pairs(const int32_t* rows, int64_t n, int32_t* out, void* stream) {
  HREC_REQUIRE(n >= 0 && out, "rows_descending_pairs: bad argument");
  hipStream_t s = as_stream(stream);
  if (hipMemsetAsync(out, 0, sizeof(int32_t), s) != hipSuccess) return check_launch("rows_descending_pairs: memset");
  if (n < 2) return HREC_OK;
  HREC_REQUIRE(rows, "rows_descending_pairs: null rows");
  hipLaunchKernelGGL(descent_kernel<int32_t>, dim3(grid_for(n)), dim3(256), 0, s, rows, n, out);
  return check_launch("descent_kernel");
}

extern "C" int hrec_coo_to_csr_sorted(const int32_t* rows, const int32_t* cols, const float* vals, int64_t nnz,
                                      int64_t n_rows, int64_t* indptr, int32_t* indices, float* values,
                                      void* stream) {
  HREC_REQUIRE(nnz >= 0 && nnz < 0x7fffffffll && n_rows >= 0 && n_rows < 0x7fffffffll,
               "coo_to_csr_sorted: bad shape");
  HREC_REQUIRE(indptr, "coo_to_csr_sorted: null indptr");
  hipStream_t s = as_stream(stream);
  if (nnz == 0) {
    if (hipMemsetAsync(indptr, 0, sizeof(int64_t) * (size_t)(n_rows + 1), s) != hipSuccess)
      return check_launch("coo_to_csr_sorted: memset");
    return HREC_OK;
  }
  HREC_REQUIRE(n_rows > 0 && rows && cols && vals && indices && values, "coo_to_csr_sorted: null pointer");
  HREC_REQUIRE((indices == cols) == (values == vals), "coo_to_csr_sorted: alias both outputs or neither");
  if (indices != cols)  // indices == cols, values == vals: the CSR is the input columns themselves
    hipLaunchKernelGGL(copy_entries_kernel, dim3(grid_for(nnz)), dim3(256), 0, s, cols, vals, nnz, indices, values);
  hipLaunchKernelGGL(indptr_from_sorted_kernel, dim3(grid_for(nnz / 4 + 1)), dim3(256), 0, s, rows, nnz, n_rows,
                     indptr);
  return check_launch("coo_to_csr_sorted");
}

// ------------------------------------------------------- shard layouts
// x[i] = table[x[i]] in place (the CSR/CSC column ids of an nnz-balanced
// ALS shard -> rows of the padded replicated factor buffer,
// src/als_engine.py:RowLayout). Ids outside [0, table_n) become -1 (the
// half-sweep's structured loads read those as zero rows).
namespace hrec {
__global__ __launch_bounds__(256) void remap_i32_kernel(int32_t* __restrict__ x, int64_t n,
                                                        const int32_t* __restrict__ table, int64_t table_n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int32_t v = x[i];
    x[i] = (v >= 0 && v < table_n) ? table[v] : -1;
  }
}
}  // namespace hrec

extern "C" int hrec_remap_i32(int32_t* x, int64_t n, const int32_t* table, int64_t table_n, void* stream) {
  HREC_REQUIRE(n >= 0 && table_n >= 0, "remap_i32: bad shape");
  if (n == 0) return HREC_OK;
  HREC_REQUIRE(x && table, "remap_i32: null pointer");
  int64_t grid = (n + 255) / 256;
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(remap_i32_kernel, dim3((unsigned)grid), dim3(256), 0, as_stream(stream), x, n, table, table_n);
  return check_launch("remap_i32_kernel");
}
