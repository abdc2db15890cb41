// K1 for ranks 65..256: ALS half-sweep with ONE WORKGROUP (8 waves) PER
// DESTINATION ROW — same arithmetic as the one-wave kernel in als.hip
// (Spark 3.5.1 ALS.computeFactors / NormalEquation.add / CholeskySolver
// [ext], reached from src/als_model.py:62), for factor widths kp in
// {96, 128, 192, 256} (BASELINE config c5 runs rank 256).
//
// Per row r:  A = sum_j v_j v_j^T (f64),  b = sum_j r_j v_j (f64),
//             A[d][d] += reg * n  (1.0 on padding columns),  A x = b,  x -> f32.
//
// Layout. The Gramian is NT x NT tiles of 16 x 16 (NT = kp / 16); the
// NT (NT + 1) / 2 upper tile pairs are dealt round-robin to the 8 waves
// (pair p -> wave p % 8, slot p / 8) and stay in registers for the whole row
// (v_mfma_f64_16x16x4_f64 C/D layout: row (lane >> 4) + 4 reg, column
// lane & 15). A kp = 256 Gramian is 263 KB — more than the LDS — so the
// factorisation and both substitutions also run on the register tiles.
//
// Phase 1 (Gramian): the row's ratings stream through LDS in windows of WR
// ratings: the block gathers the WR source rows (coalesced float4 loads,
// issued one window ahead), converts them once to f64 and stores them
// [WR][kp + 16] (the 16-double pad makes the two rows of a ds_read_b64 lane
// group hit disjoint banks). Every wave then feeds its tile pairs: operand of
// tile T for rating step s is v[4 s + (lane >> 4)][16 T + (lane & 15)].
// Threads t < kp accumulate b_t in f64.
//
// Phase 2 (factor): blocked right-looking LDL^T (A = U^T D U, U unit upper),
// block row J at a time: the owners write block row J to an LDS panel; each
// of up to 5 waves factors the 16 x 16 diagonal block redundantly (lanes
// 0..15) beside 48 panel columns of its own (lane per column, pivot row by a
// wave-private broadcast, 1/pivot by v_rcp_f64 + one Newton step — no square
// roots, no cross-wave barrier per pivot); U_J goes back to the panel and
// every owner of a trailing tile (K, M) applies A_KM -= U_JK^T D_J U_JM on
// the f64 matrix cores; owners of row J keep U_JK in their registers.
// Two barriers per block row (double-buffered panel).
//
// Phase 3 (solve): U^T w = b block by block (the owner of (J, J) solves its
// 16 x 16 triangle; owners of (J, K) subtract U_JK^T w_J from b_K), v = w / D,
// then U x = v from the last block up (owners of (J, M) subtract U_JM x_M
// from v_J). Spark's dppsv factors A = R^T R with R = D^(1/2) U: the same x.
#include "common.h"

#ifndef HREC_WIDE_WAVES
#define HREC_WIDE_WAVES(NT) 8
#endif
#ifndef HREC_WIDE_G
#define HREC_WIDE_G 4  // Gramian tile slots per operand-read group (reads of group g + 1 overlap group g's MFMAs)
#endif
#ifndef HREC_WIDE_BDEFER
#define HREC_WIDE_BDEFER 0  // 1 = a window's rhs accumulation runs during the next window's MFMAs (3 window buffers; measured 640 -> 645 ms per rank-256 epoch, off)
#endif
#ifndef HREC_WIDE_WR_WIDE
#define HREC_WIDE_WR_WIDE 32  // ratings per window at kp >= 192 (16: 641 ms, 32: 638 ms per rank-256 epoch) (multiple of 4; LDS: two windows of WR x (kp + 16) doubles)
#endif
#ifndef HREC_WIDE_CUT
#define HREC_WIDE_CUT 0  // timing/diagnostic builds only: 1 = Gramian only, 2 = no substitutions
#endif

namespace hrec {

#ifdef HREC_WIDE_STAMPS
// Diagnostic build only: per-phase cycle sums (s_memtime) of wave 0 of every
// block: [0] Gramian, [1] trailing updates + panel write + barrier, [2]
// panels, [3] tile staging, [4] x store; backward substitution per block:
// [5] wave 0's chain, [6] its column updates, [7] barrier.
__device__ unsigned long long g_wide_stamps[8];
#define WSTAMP_DECL unsigned long long _ws_prev = 0
#define WSTAMP(i)                                                                              \
  do {                                                                                         \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                                \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    if (threadIdx.x == 0 && (i) >= 0) atomicAdd(&g_wide_stamps[(i) >= 0 ? (i) : 0], _t - _ws_prev); \
    _ws_prev = _t;                                                                             \
  } while (0)
#else
#define WSTAMP_DECL
#define WSTAMP(i) \
  do {            \
  } while (0)
#endif

typedef double wd4 __attribute__((ext_vector_type(4)));

__device__ float wide_sbuf_load_f1(hrec_rsrc_t rsrc, int vindex, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.struct.buffer.load.f32");

// Waves per row: 8 for kp <= 128; 16 for kp >= 192, so that each wave's
// share of the register-resident Gramian tiles (<= 9 x 8 VGPRs) fits the
// 128 VGPRs of a 1024-thread block.
template <int NT>
struct WideShape {
  static constexpr int WAVES = HREC_WIDE_WAVES(NT);
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int KP = 16 * NT;
  static constexpr int NPAIR = NT * (NT + 1) / 2;
  static constexpr int SLOTS = (NPAIR + WAVES - 1) / WAVES;
  static constexpr int LD = KP + 16;                     // f64 row stride of windows and panels
  static constexpr int WR = KP >= 192 ? HREC_WIDE_WR_WIDE : 32;  // ratings per window
  static constexpr int WIN = WR * LD;                    // doubles per window buffer
  static constexpr int PANEL = 16 * LD;                  // doubles per panel buffer
  static constexpr int BUF = WIN > PANEL ? WIN : PANEL;  // windows and panels share two buffers
  static constexpr int F4 = WR * KP / 4;                 // float4 loads per window
  static constexpr int F4_PER_T = (F4 + THREADS - 1) / THREADS;
};

// Pair p (row-major over the upper tile triangle) -> (I, J).
template <int NT>
__device__ __forceinline__ void pair_ij(int p, int& I, int& J) {
  int i = 0;
#pragma unroll
  for (int r = 0; r < NT; ++r) {
    const int len = NT - r;
    if (p >= len && i == r) {
      p -= len;
      i = r + 1;
    }
  }
  I = i;
  J = i + p;
}

__device__ __forceinline__ double wbcast(double v, int src) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)x, src);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// A double moved across lanes by one DPP pattern (two 32-bit v_mov_dpp).
template <int CTRL>
__device__ __forceinline__ double dpp64(double x) {
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(v >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Backward substitution: the wave that runs block M's chain also applies its
// own tiles of column M + 1 right after it (on the critical path), so pick,
// per block, the wave owning the fewest such tiles (I, M + 1), I < M
// (pair p -> wave p % WAVES). Packed 3 bits per block at compile time.
template <int NT, int WAVES>
constexpr unsigned long long chain_waves_packed() {
  unsigned long long packed = 0;
  for (int M = 0; M < NT; ++M) {
    int best = 0, bestc = 1 << 30;
    for (int w = 0; w < WAVES; ++w) {
      int c = 0;
      for (int I = 0; M + 1 < NT && I < M; ++I) {
        const int p = I * NT - I * (I - 1) / 2 + (M + 1 - I);
        if (p % WAVES == w) ++c;
      }
      if (c < bestc) {
        bestc = c;
        best = w;
      }
    }
    packed |= (unsigned long long)best << (3 * M);
  }
  return packed;
}

template <int NT>
__global__ __launch_bounds__(WideShape<NT>::THREADS) void als_half_sweep_wide_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices, const float* __restrict__ values,
    int64_t n_rows, const float* __restrict__ src, int64_t n_src, int k, double reg, float* __restrict__ dst) {
  using S = WideShape<NT>;
  constexpr int KP = S::KP, LD = S::LD, WR = S::WR, kWideWaves = S::WAVES, kWideThreads = S::THREADS;
  // window buffers: NB = 3 rotates current / next / previous window (the
  // previous one's rhs accumulation overlaps the current one's MFMAs);
  // phase 2 uses buffers 0, 1 as its double-buffered panel
  constexpr int NB = HREC_WIDE_BDEFER ? 3 : 2;
  __shared__ __attribute__((aligned(16))) double buf[NB][S::BUF];
  __shared__ double bsh[KP];      // b, then w (forward), then v / x
  __shared__ double dsh[KP];      // pivots D
  __shared__ double rdsh[KP];     // 1 / D
  __shared__ double xsh[KP];      // x blocks (backward)
  __shared__ float rsh[NB][WR];   // ratings of the windows in buf
  __shared__ __attribute__((aligned(16))) double tri[kWideWaves][64];  // per-wave scratch: the panel's two 32-entry pivot-row buffers
  __shared__ double udg[16 * 17];              // U_JJ of the current block row
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sub = lane >> 4, col = lane & 15;
  const int64_t row = blockIdx.x;
  const int64_t beg = indptr[row], end = indptr[row + 1];
  float* __restrict__ out = dst + row * KP;
  if (end == beg) {
    if (tid < KP) out[tid] = 0.f;
    return;
  }
  const int64_t n = end - beg;

  // ---------------------------------------------------------------- phase 1
  WSTAMP_DECL;
  WSTAMP(-1);
  wd4 acc[S::SLOTS];
  int pij[S::SLOTS];  // (I | J << 8) of each slot's tile pair, -1 = none (wave-uniform)
#pragma unroll
  for (int s = 0; s < S::SLOTS; ++s) {
    acc[s] = wd4{0.0, 0.0, 0.0, 0.0};
    const int p = s * kWideWaves + w;
    int I = 0, J = 0;
    pair_ij<NT>(p, I, J);
    pij[s] = __builtin_amdgcn_readfirstlane(p < S::NPAIR ? (I | (J << 8)) : -1);
  }
  double bacc = 0.0;  // b[tid] for tid < KP
  float4 ld[S::F4_PER_T];
  float lr = 0.f;     // this thread's rating slot (tid < WR)
  const int nwin = (int)((n + WR - 1) / WR);
  // Two-stage window prefetch: the source-row indices of window w + 2 are
  // loaded while window w computes, the rows (and ratings) of window w + 1
  // from indices already in registers — so no window start waits on a
  // dependent index -> row round trip. Loads are unconditional (clamped
  // addresses, results selected), so no branch splits the issue.
  // Every validity test is applied where the loaded value is consumed (the
  // rows at the conversion, the indices when the rows are issued), so no
  // wait follows a load.
  int ixn[S::F4_PER_T];  // raw source rows of the next window's float4 slots (kUniRow: slot lane & 1)
  bool okq[S::F4_PER_T];  // slot q of the window in `ld` holds a real row
  bool okr = false;       // the rating in `lr` is real
  // indices / ratings of this row through buffer resources based at the
  // row's first entry (32-bit element offsets in VGPRs, the 64-bit bases in
  // SGPRs: no per-lane 64-bit address pairs)
  const hrec_rsrc_t irs = rows_rsrc(indices, beg, 4, end);
  const hrec_rsrc_t vrs = rows_rsrc(values, beg, 4, end);
  const int n32 = (int)n;  // ratings of this row (< 2^31)
  // kp 256 at 8 waves: a float4 slot's window row is wave-uniform (64 float4
  // per row), so the index loads need no per-thread row arithmetic
  constexpr bool kUniRow = KP / 4 == 64 && S::F4 % kWideThreads == 0;
  auto load_idx = [&](int win, int (&ix)[S::F4_PER_T]) {
#pragma unroll
    for (int q = 0; q < S::F4_PER_T; ++q) {
      int p;
      if constexpr (kUniRow) {
        // one source row per wave and slot (row w + 8 q of the window): lane
        // l loads slot l % F4_PER_T's index, read back by v_readlane when the rows
        // are issued (a per-lane address keeps the value in a VGPR, so
        // nothing waits for it here)
        if (q > 0) break;
        p = win * WR + w + (kWideThreads / 64) * (__lane_id() % S::F4_PER_T);
      } else {
        const int e = tid + q * kWideThreads;
        p = win * WR + (e < S::F4 ? e / (KP / 4) : 0);
      }
      ix[q] = __float_as_int(wide_sbuf_load_f1(irs, p < n32 ? p : n32 - 1, 0, 0, 0));
    }
  };
  auto load_rows = [&](int win, const int (&ix)[S::F4_PER_T]) {
#pragma unroll
    for (int q = 0; q < S::F4_PER_T; ++q) {
      int c4, p, iq = ix[q];
      bool inw;
      if constexpr (kUniRow) {
        c4 = __lane_id();
        p = win * WR + w + (kWideThreads / 64) * q;
        inw = true;  // ix[q]: slot q's index, already wave-uniform
      } else {
        const int e = tid + q * kWideThreads;
        c4 = e % (KP / 4);
        p = win * WR + (e < S::F4 ? e / (KP / 4) : 0);
        inw = e < S::F4;
      }
      okq[q] = inw && p < n32 && iq >= 0 && iq < n_src;
      ld[q] = *reinterpret_cast<const float4*>(src + (int64_t)(okq[q] ? iq : 0) * KP + 4 * c4);
    }
    // the ratings: consumed at the window's conversion, so one window ahead
    const int l = kUniRow ? __lane_id() : tid;  // the rating slots are lanes 0..WR-1 of wave 0
    const int pr = win * WR + (l < WR ? l : 0);
    lr = wide_sbuf_load_f1(vrs, pr < n32 ? pr : n32 - 1, 0, 0, 0);
    okr = tid < WR && win * WR + l < n32;
  };
  auto load_window = [&](int win) {  // window `win` now (prologue)
    int ix[S::F4_PER_T], iu[S::F4_PER_T];
    load_idx(win, ix);
#pragma unroll
    for (int q = 0; q < S::F4_PER_T; ++q) iu[q] = kUniRow ? __builtin_amdgcn_readlane(ix[0], q) : ix[q];
    load_rows(win, iu);
  };
  auto store_window = [&](int b) {
#pragma unroll
    for (int q = 0; q < S::F4_PER_T; ++q) {
      const int e = tid + q * kWideThreads;
      if (e < S::F4) {
        const int r = e / (KP / 4), c4 = e % (KP / 4);
        double* d = &buf[b][r * LD + 4 * c4];
        const float4 t = okq[q] ? ld[q] : make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<double2*>(d) = make_double2((double)t.x, (double)t.y);
        *reinterpret_cast<double2*>(d + 2) = make_double2((double)t.z, (double)t.w);
      }
    }
    if (tid < WR) rsh[b][tid] = okr ? lr : 0.f;
  };
  load_window(0);
  if (nwin > 1) load_idx(1, ixn);
  store_window(0);
  __syncthreads();
  // b over one window's ratings (threads t < kp, ratings in order)
  auto rhs_window = [&](int b) {
    if (tid < KP) {
#pragma unroll 4
      for (int r = 0; r < WR; ++r) bacc = fma((double)rsh[b][r], buf[b][r * LD + tid], bacc);
    }
  };
  int cb = 0;  // buffer of window `win`
  for (int win = 0; win < nwin; ++win) {
    const int nb = cb + 1 == NB ? 0 : cb + 1;  // next window's buffer
    if (win + 1 < nwin) {  // wave-uniform
      // the index loads first: a value reloaded from scratch on the way
      // (vmcnt counts in issue order) then waits for them, not for the rows
      // (kp 256: the per-slot indices leave the VGPR by v_readlane first, so
      // the next index load reuses its register — no loop-carried copy that
      // would wait for it)
      int ixc[S::F4_PER_T];
#pragma unroll
      for (int q = 0; q < S::F4_PER_T; ++q) ixc[q] = kUniRow ? __builtin_amdgcn_readlane(ixn[0], q) : ixn[q];
      if (win + 2 < nwin) load_idx(win + 2, ixn);
      load_rows(win + 1, ixc);
    }
    // HREC_WIDE_BDEFER: the previous window's b (buffer nb + 1 mod 3) before
    // this window's MFMAs — on waves 0..3, whose SIMD partners (waves 4..7)
    // keep the matrix pipe busy meanwhile — instead of after them on the
    // path to the barrier
    if (HREC_WIDE_BDEFER && win > 0) rhs_window(nb + 1 == NB ? 0 : nb + 1);
    const double* wb = buf[cb];
#pragma unroll 1
    for (int st = 0; st < WR / 4; ++st) {
      const double* vrow = wb + (4 * st + sub) * LD + col;
      // No per-slot branch (a slot without a pair accumulates tile (0, 0)
      // into a register nobody reads). Slots go in groups of G: the operand
      // reads of group g + 1 are issued before the MFMAs of group g, so the
      // LDS latency hides behind G MFMAs (64 cycles each).
      constexpr int G = HREC_WIDE_G, NG = (S::SLOTS + G - 1) / G;
      double ra[2][G], rb[2][G];
      auto rd = [&](int g, int bsel) {
#pragma unroll
        for (int j = 0; j < G; ++j) {
          const int s = g * G + j;
          if (s < S::SLOTS) {
            const int q = pij[s] < 0 ? 0 : pij[s];
            ra[bsel][j] = vrow[16 * (q & 255)];
            rb[bsel][j] = vrow[16 * (q >> 8)];
          }
        }
      };
      rd(0, 0);
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        if (g + 1 < NG) rd(g + 1, (g + 1) & 1);
#pragma unroll
        for (int j = 0; j < G; ++j) {
          const int s = g * G + j;
          if (s < S::SLOTS) acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(ra[g & 1][j], rb[g & 1][j], acc[s], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // (the last window's b before the barrier: phase 2 reuses buffers 0, 1)
    if (!HREC_WIDE_BDEFER || win + 1 == nwin) rhs_window(cb);
    if (win + 1 < nwin) store_window(nb);
    __syncthreads();
    cb = nb;
  }
  // lambda = numExplicits * regParam on the diagonal (1.0 on padding columns)
  const double lambda = (double)n * reg;
#pragma unroll
  for (int s = 0; s < S::SLOTS; ++s) {
    if (pij[s] >= 0) {
      const int I = pij[s] & 255, J = pij[s] >> 8;
      if (I == J) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (sub + 4 * r == col) acc[s][r] += (16 * I + col < k) ? lambda : 1.0;
      }
    }
  }
  if (tid < KP) bsh[tid] = bacc;
#if HREC_WIDE_CUT == 1
  {
    double t = bacc;
#pragma unroll
    for (int s = 0; s < S::SLOTS; ++s) t += acc[s][0] + acc[s][1] + acc[s][2] + acc[s][3];
    if (tid < KP) out[tid] = (float)t;
    return;
  }
#endif

  WSTAMP(0);
  // ---------------------------------------------------------------- phase 2
  // (a) owners of block row J -> panel rows 0..15
  auto write_panel = [&](int J) {
    double* P = buf[J & 1];
#pragma unroll
    for (int s = 0; s < S::SLOTS; ++s) {
      if (pij[s] >= 0) {
        const int I = pij[s] & 255, K = pij[s] >> 8;
        if (I == J) {
#pragma unroll
          for (int r = 0; r < 4; ++r) P[(sub + 4 * r) * LD + 16 * K + col] = acc[s][r];
        }
      }
    }
  };
  // (b) panel: wave w < n_act takes the diagonal block (lanes 0..15,
  //     redundantly) and 48 columns beyond it (lanes 16..63)
  auto panel = [&](int J) {
    double* P = buf[J & 1];
    const int rest = KP - 16 * (J + 1);
    const int n_act = rest > 0 ? (rest + 47) / 48 : 1;
    if (HREC_WIDE_CUT != 3 && w < n_act) {
      // lane per column, column in registers, pivot loop rolled (a[] is only
      // ever indexed by compile-time m; a[i] comes out through a select
      // chain): lanes 0..15 of every active wave hold the diagonal block
      // (read-only in P: each wave factors it privately, no cross-wave
      // barrier per pivot), lanes 16..63 one panel column each.
      const int c = lane < 16 ? 16 * J + lane : 16 * (J + 1) + 48 * w + (lane - 16);
      const bool own = c < KP;
      const double* pc = P + (own ? c : KP + (lane & 15));  // idle lanes read pad columns
      double a[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) a[m] = pc[m * LD];
      if (lane < 32) tri[w][16 + lane + 16 * (lane >> 4)] = 0.0;  // entries 16..31 of both buffers
      wave_sync_lds();
#pragma unroll 1
      for (int i = 0; i < 16; ++i) {
        // a[] is kept shifted: a[0] is always the column's row 16 J + i, so
        // the rolled loop indexes registers at compile time only
        const double ai = a[0];
        const double piv = wbcast(ai, i);  // lane i: column 16 J + i, row 16 J + i
        const double r0 = __builtin_amdgcn_rcp(piv);
        const double rp = fma(r0, fma(-piv, r0, 1.0), r0);
        const double ut = ai * rp;  // U[16 J + i][c]
        // pivot row inside the diagonal block: 32-entry buffers whose upper
        // half stays zero, so the shifted reads below never leave them
        double* cbw = tri[w] + 32 * (i & 1);
        if (lane < 16) cbw[lane] = ai;
        if (own && lane >= 16) P[i * LD + c] = ut;  // the panel column's row i becomes U
        if (w == 0 && lane < 16) udg[i * 17 + lane] = lane > i ? ut : (lane == i ? 1.0 : 0.0);
        if (w == 0 && lane == i) {
          dsh[16 * J + i] = piv;
          rdsh[16 * J + i] = rp;
        }
        wave_sync_lds();
        double u[15];
#pragma unroll
        for (int j = 0; j < 15; ++j) u[j] = cbw[i + 1 + j];
#pragma unroll
        for (int j = 0; j < 15; ++j) a[j] = fma(-u[j], ut, a[j + 1]);
      }
      // forward substitution of block J (U_JJ^T w_J = b_J, b_J final: every
      // earlier block already subtracted its part) by wave 0, which has just
      // written U_JJ to udg; v_J = w_J / D
      if (w == 0) {
        wave_sync_lds();
        double tc[16];  // column `lane` of U_JJ
#pragma unroll
        for (int q = 0; q < 16; ++q) tc[q] = udg[q * 17 + col];
        double bi = lane < 16 ? bsh[16 * J + lane] : 0.0;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const double wq = wbcast(bi, q);
          if (lane > q && lane < 16) bi = fma(-tc[q], wq, bi);
        }
        if (lane < 16) {
          xsh[16 * J + lane] = bi;                        // w_J
          bsh[16 * J + lane] = bi * rdsh[16 * J + lane];  // v_J
        }
      }
    }
  };
  // b_K -= U_JK^T w_J for every later column, one thread per column (the
  // panel still holds U_J)
  auto rhs_upd = [&](int J) {
    const double* P = buf[J & 1];
    if (tid < KP - 16 * (J + 1)) {
      const int cc = 16 * (J + 1) + tid;
      double part = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) part = fma(P[q * LD + cc], xsh[16 * J + q], part);
      bsh[cc] -= part;
    }
  };
  // (c) trailing update A_KM -= U_JK^T D_J U_JM of the tiles with kstop < K
  // <= kmax. Slot rows K grow with the slot index, so they are a suffix of
  // the slots (minus rows above kmax): walk it from the end, reading the next
  // slot's panel operands before this slot's four MFMAs.
  auto trail = [&](int J, int kstop, int kmax) {
    if (HREC_WIDE_CUT == 4) return;
    const double* P = buf[J & 1];
    const double* dj = dsh + 16 * J;
    auto opnd = [&](int s, double (&ua)[4], double (&ub)[4]) {
      const int q0 = pij[s] < 0 ? 0 : pij[s];
      const int K = q0 & 255, M = q0 >> 8;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int q = 4 * kk + sub;
        ua[kk] = -P[q * LD + 16 * K + col] * dj[q];
        ub[kk] = P[q * LD + 16 * M + col];
      }
    };
    double ua[4], ub[4];
    opnd(S::SLOTS - 1, ua, ub);
#pragma unroll
    for (int s = S::SLOTS - 1; s >= 0; --s) {
      const int K = pij[s] & 255;
      if (pij[s] >= 0 && K <= kstop) break;  // wave-uniform
      double ca[4], cbv[4];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        ca[kk] = ua[kk];
        cbv[kk] = ub[kk];
      }
      if (s > 0) opnd(s - 1, ua, ub);
      if (pij[s] >= 0 && K <= kmax) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
          acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(ca[kk], cbv[kk], acc[s], 0, 0, 0);
      }
    }
  };
  // owners of row J take U_JK (the panel) / U_JJ (udg)
  auto take_u = [&](int J) {
    if (HREC_WIDE_CUT == 4) return;
    const double* P = buf[J & 1];
#pragma unroll
    for (int s = 0; s < S::SLOTS; ++s) {
      if (pij[s] >= 0 && (pij[s] & 255) == J) {
        const int M = pij[s] >> 8;
        if (M == J) {
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[s][r] = udg[(sub + 4 * r) * 17 + col];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[s][r] = P[(sub + 4 * r) * LD + 16 * M + col];
        }
      }
    }
  };
#pragma unroll 1
  for (int J = 0; J < NT; ++J) {
    write_panel(J);
    __syncthreads();
    WSTAMP(1);
    panel(J);
    __syncthreads();
    WSTAMP(2);
    rhs_upd(J);  // beside the trailing MFMAs below
    trail(J, J, NT);
    take_u(J);
  }
  __syncthreads();

#if HREC_WIDE_CUT == 2 || HREC_WIDE_CUT == 3 || HREC_WIDE_CUT == 4
  {
    double t = 0.0;
#pragma unroll
    for (int s = 0; s < S::SLOTS; ++s) t += acc[s][0] + acc[s][1] + acc[s][2] + acc[s][3];
    if (tid < KP) out[tid] = (float)t;
    return;
  }
#endif
  WSTAMP(3);
  // ---------------------------------------------------------------- phase 3
  // Backward substitution U x = v (v in bsh; the forward one ran inside the
  // factorisation), one barrier per block: one wave (per block the one with
  // the fewest own column updates) runs the dependent chain
  // x_M = U_MM^-1 (v_M - U_M,M+1 x_M+1) from the diagonal and
  // super-diagonal tiles staged in the (now free) window buffers, while the
  // owners of the other tiles of column M + 1 apply U_I,M+1 x_M+1 to the
  // rows I < M. Each row still receives its column contributions in
  // descending column order and every partial sum keeps its 16-lane
  // butterfly order, so x is bit-identical to the two-barrier form.
  double* const Dg = &buf[0][0];     // tile (M, M) at Dg + 272 M, row-major 16 x 17
  double* const Sd = Dg + 272 * NT;  // tile (M - 1, M) at Sd + 272 M
  static_assert(2 * 272 * NT <= 2 * S::BUF, "diagonal + super-diagonal tiles fit the window buffers");
#pragma unroll
  for (int s = 0; s < S::SLOTS; ++s) {
    if (pij[s] >= 0) {
      const int I = pij[s] & 255, K = pij[s] >> 8;
      if (K == I || K == I + 1) {
        double* T = (K == I ? Dg : Sd) + 272 * K;
#pragma unroll
        for (int r = 0; r < 4; ++r) T[(sub + 4 * r) * 17 + col] = acc[s][r];
      }
    }
  }
  __syncthreads();
  static_assert(kWideWaves <= 8 && 3 * NT <= 64, "chain-wave table: 3 bits per block");
  constexpr unsigned long long kChain = chain_waves_packed<NT, kWideWaves>();
#pragma unroll 1
  for (int M = NT - 1; M >= 0; --M) {
    if (w == (int)((kChain >> (3 * M)) & 7)) {
      const double* Td = Dg + 272 * M + col * 17;  // row `lane` of U_MM
      double tr[16];  // loaded first: their LDS latency hides behind the GEMV below
#pragma unroll
      for (int q = 0; q < 16; ++q) tr[q] = Td[q];
      double bi = lane < 16 ? bsh[16 * M + lane] : 0.0;
      if (M + 1 < NT) {  // v_M -= U_M,M+1 x_M+1 (lane i < 16: row i; butterfly order)
        const double* T = Sd + 272 * (M + 1) + col * 17;
        const double* xm = xsh + 16 * (M + 1);
        // products rounded on their own (no contraction into the adds), the
        // pairwise tree built as the products arrive (few live registers)
        auto pr = [&](int q) { return __dmul_rn(T[q], xm[q]); };
        auto quad = [&](int q) { return __dadd_rn(__dadd_rn(pr(q), pr(q + 1)), __dadd_rn(pr(q + 2), pr(q + 3))); };
        const double lo = __dadd_rn(quad(0), quad(4));
        const double hi = __dadd_rn(quad(8), quad(12));
        bi = __dsub_rn(bi, __dadd_rn(lo, hi));
      }
#pragma unroll
      for (int q = 15; q >= 0; --q) {
        const double xq = wbcast(bi, q);
        if (lane < q) bi = fma(-tr[q], xq, bi);
      }
      if (lane < 16) xsh[16 * M + lane] = bi;
    }
    WSTAMP(5);
    if (M + 1 < NT) {
#pragma unroll
      for (int s = 0; s < S::SLOTS; ++s) {
        if (pij[s] >= 0) {
          const int I = pij[s] & 255, K = pij[s] >> 8;
          if (K == M + 1 && I < M) {  // v_I -= U_I,M+1 x_M+1
            const double xm = xsh[16 * K + col];
            double part[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              part[r] = acc[s][r] * xm;
              // 16-lane butterfly by DPP moves (no LDS round trips): swaps
              // inside quads, then the half-row and row mirrors — lane 0
              // (the only reader) adds exactly the partial sums the xor
              // butterfly would (the mirrored lanes hold the same bits)
              part[r] += dpp64<0xB1>(part[r]);   // quad_perm [1,0,3,2]
              part[r] += dpp64<0x4E>(part[r]);   // quad_perm [2,3,0,1]
              part[r] += dpp64<0x141>(part[r]);  // row_half_mirror
              part[r] += dpp64<0x140>(part[r]);  // row_mirror
            }
            if (col == 0) {
#pragma unroll
              for (int r = 0; r < 4; ++r) bsh[16 * I + sub + 4 * r] -= part[r];
            }
          }
        }
      }
    }
    WSTAMP(6);
    __syncthreads();
    WSTAMP(7);
  }
  if (tid < KP) out[tid] = (float)xsh[tid];
  WSTAMP(4);
}

}  // namespace hrec

using namespace hrec;

#ifdef HREC_WIDE_STAMPS
extern "C" int hrec_debug_wide_stamps(unsigned long long* host_out, int reset) {
  if (hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_wide_stamps), sizeof(g_wide_stamps)) != hipSuccess) return -2;
  if (reset) {
    unsigned long long z[8] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_wide_stamps), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 0;
}
#endif

int hrec_als_half_sweep_wide(const int64_t* indptr, const int32_t* indices, const float* values, int64_t n_rows,
                             const float* src_factors, int64_t n_src, int k, int kp, double reg_param,
                             float* dst_factors, void* stream) {
  const dim3 grid((unsigned)n_rows);
  hipStream_t s = as_stream(stream);
#define HREC_WIDE(NT)                                                                                        \
  hipLaunchKernelGGL((als_half_sweep_wide_kernel<NT>), grid, dim3(WideShape<NT>::THREADS), 0, s, indptr, indices, values, n_rows, \
                     src_factors, n_src, k, reg_param, dst_factors)
  switch (kp) {
    case 96: HREC_WIDE(6); break;
    case 128: HREC_WIDE(8); break;
    case 192: HREC_WIDE(12); break;
    default: HREC_WIDE(16); break;
  }
#undef HREC_WIDE
  return check_launch("als_half_sweep_wide_kernel");
}
