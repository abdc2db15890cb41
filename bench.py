"""Headline benchmark: ALS epochs/sec (+ scored user-item pairs/sec) at rank 64.

Workload (BASELINE.json configs[1], SURVEY §8d "c2"): synthetic 1,000,000 users
x 100,000 items at 0.5 % density (nnz ~ 5.0e8, ratings 0..18), rank 64,
reg 0.1. One step = one ALS epoch = item half-sweep + user half-sweep
(Spark's iteration order), generated and kept on the device (inputs resident
in HBM before the timed region). With N ranks, users and items are
row-sharded and the factors replicated by RCCL all-gathers after each
half-sweep; the total work is fixed (scaling "strong"). `--gpus N` without
torchrun starts the N rank processes itself (torch.distributed.run, before
any GPU call). With 8 or more ranks the line also carries `als_c3`
(BASELINE configs[2]: 10M x 1M at 1 %, rank 64, user-sharded with chunked
RCCL all-gathers); `--config c3` makes c3 the headline (8 ranks required).

Also measured in the same run (not the headline value):
  * scoring: B users x all items, JVM-exact ALS dot + stable top-5 on the
    device (pairs scored and consumed by top-k per second);
  * roofline of the dominant kernel (als_half_sweep_f64_kernel), timed with
    HIP events on the stream it is launched on;
  * cpu_baseline: the C oracle (Spark ALS restated, OpenMP) on rank 0 over a
    bounded row sample of the same matrix, extrapolated to one epoch;
  * tt_scoring_c4 (BASELINE configs[3]): two-tower d = 128, 50M candidate
    items split across the ranks, a batch of users ranked top-5 by the fused
    matrix-core dot + top-k (f32 = Keras numerics, and bf16), C3 merge.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hybrid-als-twotower-recommender_amd"))
sys.path.insert(0, ROOT)

from src import _hrec, synthetic  # noqa: E402
from src.als_engine import DeviceALS, RowLayout, shard_range  # noqa: E402
from src.recommend import CapturedRecommend, ShardedRecommender, ShardedScorer  # noqa: E402
from src.tt_engine import DeviceTwoTower  # noqa: E402

METRIC = "ALS epochs/sec + scored user-item pairs/sec at rank=64, 1/2/4/8 MI355X"
F64_MFMA_PEAK_TFLOPS = 78.6  # AMD MI355X spec (FP64 matrix); not in MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
F32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: f32-input MFMA = f32 VALU peak (64 flop/clk/SIMD)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16
# JVM-exact scoring forbids FMA: one v_pk_mul_f32 + one v_pk_add_f32 per 2
# products -> half the 157.3 TF FMA rate (measured issue rate 60 T)
F32_VALU_MULADD_TFLOPS = 78.6

CONFIGS = {
    "c2": dict(users=1_000_000, items=100_000, density=0.005, rank=64),
    "c2s": dict(users=100_000, items=20_000, density=0.005, rank=64),  # quick check
    # BASELINE configs[2]: one rank's shard (~200 GB of CSR + CSC) is sized
    # for 8 GPUs
    "c3": dict(users=10_000_000, items=1_000_000, density=0.01, rank=64, min_world=8, layout="equal"),
}
# HREC_BENCH_C3_REHEARSAL="W:f": c3's flow at f x its users and items from W
# ranks (the one-GPU gloo rehearsal of the 8-GPU sub-line; labelled in the line)
if os.environ.get("HREC_BENCH_C3_REHEARSAL"):
    _w, _f = os.environ["HREC_BENCH_C3_REHEARSAL"].split(":")
    CONFIGS["c3"].update(users=int(CONFIGS["c3"]["users"] * float(_f)), items=int(CONFIGS["c3"]["items"] * float(_f)),
                         min_world=int(_w), rehearsal=True)


def algo_flops(nnz, n_dst, k):
    """symmetric rank-1 Gramian + rhs per rating, Cholesky + 2 solves per row."""
    return nnz * (k * (k + 1) + 2 * k) + n_dst * (k ** 3 / 3 + 2 * k * k)


def algo_bytes(nnz, n_dst, k):
    """index + value + one gathered f32 factor row per rating, indptr, dst write."""
    return nnz * (4 + 4 + 4 * k) + (n_dst + 1) * 8 + n_dst * k * 4


def ev_time(fn, reps, stream):
    """Average ms of fn() over reps, HIP events on the stream fn launches on."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def roofline(bound, work, ms, peak, unit, kernel, **extra):
    """work = algorithmic flops or bytes of ONE launch of `kernel`; ms = its
    average launch duration (HIP events)."""
    ach = work / (ms / 1e3) / (1e12 if unit == "TFLOP/s" else 1e9)
    out = {"kernel": kernel, "bound": bound, "achieved": ach, "peak": peak, "unit": unit, "frac": ach / peak,
           "avg_launch_ms": ms, ("algorithmic_flops" if unit == "TFLOP/s" else "algorithmic_bytes"): work}
    out.update(extra)
    return out


def time_recommend(rec, hu, uvec, world, reps=20):
    """Seconds per batch (max over ranks): at W = 1 the batch replayed as one
    HIP graph (CapturedRecommend), at W > 1 eager (the C2/C3 collectives run
    between the kernels). Returns (seconds, eager seconds or None)."""
    def run_timed(fn):
        for _ in range(2):
            fn()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        ht = torch.tensor([(time.perf_counter() - h0) / reps], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(ht, op=dist.ReduceOp.MAX)
        return float(ht.item())

    eager = run_timed(lambda: rec.recommend(hu, uvec, False, 5))
    if world > 1:
        return eager, None
    cap = CapturedRecommend(rec, hu, uvec, False, 5)
    ei, ev = rec.recommend(hu, uvec, False, 5)
    gi, gv = cap()
    if not (torch.equal(ei, gi) and torch.equal(ev, gv)):
        raise RuntimeError("captured recommend differs from eager")
    return run_timed(cap), eager


def recommend_line_timing(hs_graph, hs_eager):
    """ms_per_batch = the faster of graph replay / eager launch (both timed)."""
    if hs_eager is None:
        return hs_graph, "eager (W > 1: collectives between kernels)"
    if hs_graph < hs_eager:
        return hs_graph, "one HIP graph per batch (CapturedRecommend)"
    return hs_eager, "eager launches (HIP-graph replay measured no faster)"


def hybrid_stages(rec, hu, uvec, top_k, reps, stream):
    """W = 1: each step of ShardedRecommender.recommend timed on its own
    (HIP events), with the roofline of each; the dominant one is the line's
    roofline. Same calls recommend() makes, in the same order."""
    o = rec.ops
    B, N = int(hu.shape[0]), rec.n_local
    if (rec.precision == "exact" and getattr(rec, "pruned_exact", False) and top_k <= _hrec.EXACT_MAX_K
            and B >= 8):
        # exact path without score matrices (csrc/hybrid_exact.hip): phase 1
        # (split-bf16 bound GEMMs of both models, no stores) + the exact
        # extremes; then the group bounds, seeds and the live groups rescored
        # by the exact chains, stable top-k
        hx = o.hybrid_exact(rec.U, hu, uvec, rec.exact_items, top_k)
        a_mm, t_mm = hx.minmax()
        d, dk = int(rec.iv.shape[1]), hx.dk
        G = -(-N // 32)
        op_b = 2.0 * 2 * 2.0 * dk * N  # both models' split operands (hi + lo bf16) read once
        st = [("hybrid_exact_minmax (split-bf16 bound GEMMs of both models, dk %d, no score stores; exact extremes "
               "of the candidate groups)" % dk, hx.minmax,
               dict(bound="hbm", work=op_b, peak=HBM_PEAK_GBS, unit="GB/s", mfma_flops=2 * 3 * 2.0 * dk * B * N))]
        hx.topk(a_mm, t_mm, False, rec.offset)
        n_ext, n_top, every = hx.counts()
        live = float(n_top.double().sum())
        # phase 2's bytes: every user's group records + the f32 item rows of
        # both models of its live groups (the exact chains' inputs)
        p2_b = 16.0 * B * G + live * 32 * 4.0 * (rec.k + d)
        st.append(("hybrid_exact_topk (group bounds, seeds, live groups rescored by the exact chains, stable "
                   "top-k)", lambda: hx.topk(a_mm, t_mm, False, rec.offset),
                   dict(bound="hbm", work=p2_b, peak=HBM_PEAK_GBS, unit="GB/s")))
        out = []
        for name, fn, rf in st:
            fn()
            ms = ev_time(fn, reps, stream)
            r = roofline(rf["bound"], rf["work"], ms, rf["peak"], rf["unit"], name)
            if "mfma_flops" in rf:
                tf = rf["mfma_flops"] / (ms * 1e-3) / 1e12
                r["mfma_view"] = {"achieved": tf, "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                                  "frac": tf / BF16_MFMA_PEAK_TFLOPS}
            out.append(r)
        local_ms = ev_time(lambda: hx.local(False, rec.offset), reps, stream)
        n_ext, n_top, every = hx.counts()
        tot = sum(r["avg_launch_ms"] for r in out)
        item_b = 4.0 * (rec.k + d) * N  # the reference's inputs: both models' f32 item rows, once
        dom = max(out, key=lambda r: r["avg_launch_ms"])
        return dict(dom, stages=out, one_shard_call_ms=local_ms, every_group_rescored=bool(every),
                    groups_per_user={"total": G, "extremes_mean": float(n_ext.double().mean()),
                                     "topk_mean": float(n_top.double().mean()), "topk_max": int(n_top.max())},
                    batch_view={"ms": tot, "algorithmic_bytes": item_b,
                                "note": "both models' f32 item rows once (the materialised path's inputs) / both "
                                        "phases' time",
                                "achieved": item_b / (tot * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": item_b / (tot * 1e-3) / 1e9 / HBM_PEAK_GBS})
    if rec.precision == "exact":
        als = o.als_scores(rec.U, hu, rec.Vt, N, rec.k)
        tt = o.tt_scores(uvec, rec.iv)
        d = rec.iv.shape[1]
        st = [("als_score (JVM-exact f32 mul+add, no FMA)",
               lambda: o.als_scores(rec.U, hu, rec.Vt, N, rec.k),
               dict(bound="valu", work=2.0 * rec.k * B * N, peak=F32_VALU_MULADD_TFLOPS, unit="TFLOP/s")),
              ("tt_score (f32 MFMA Dot)", lambda: o.tt_scores(uvec, rec.iv),
               dict(bound="mfma", work=2.0 * d * B * N, peak=F32_MFMA_PEAK_TFLOPS, unit="TFLOP/s"))]
    elif getattr(rec, "pruned", False) and top_k <= _hrec.PRUNE_MAX_K:
        # pruned bf16 path (csrc/hybrid_prune.hip): no score matrix; phase 1
        # reads both models' item operands, phase 2 the heavier model's
        hp = o.hybrid_prune(rec.U, hu, uvec, rec.V_op, rec.iv_op, top_k)
        a_mm, t_mm = hp.minmax()
        op_b = 2.0 * rec.dk * N  # one model's bf16 item operand
        st = [("hybrid_prune_minmax (both bf16 GEMMs, dk %d, no score stores: row min/max + group max slices)"
               % rec.dk, hp.minmax,
               dict(bound="hbm", work=2 * op_b, peak=HBM_PEAK_GBS, unit="GB/s", mfma_flops=2 * 2.0 * rec.dk * B * N)),
              ("hybrid_prune_topk (bound + heavier model's bf16 GEMM with survivor filter + survivors' fusion "
               "+ stable top-k)", lambda: hp.topk(a_mm, t_mm, False, rec.offset),
               dict(bound="hbm", work=op_b, peak=HBM_PEAK_GBS, unit="GB/s", mfma_flops=2.0 * rec.dk * B * N))]
        out = []
        for name, fn, rf in st:
            fn()
            ms = ev_time(fn, reps, stream)
            r = roofline(rf["bound"], rf["work"], ms, rf["peak"], rf["unit"], name)
            tf = rf["mfma_flops"] / (ms * 1e-3) / 1e12
            r["mfma_view"] = {"achieved": tf, "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                              "frac": tf / BF16_MFMA_PEAK_TFLOPS}
            out.append(r)
        fell_back = hp.fallback_taken()
        surv = hp.survivors().double()
        # the single-shard call the recommender makes at W = 1 (both phases,
        # the extremes folded into the bound launch)
        local_ms = ev_time(lambda: hp.local(False, rec.offset), reps, stream)
        tot = sum(r["avg_launch_ms"] for r in out)
        dom = max(out, key=lambda r: r["avg_launch_ms"])
        return dict(dom, stages=out, fallback_taken=fell_back, one_shard_call_ms=local_ms,
                    survivors_per_user={"mean": float(surv.mean()), "max": float(surv.max())},
                    batch_view={"ms": tot, "algorithmic_bytes": 2 * op_b,
                                "note": "no-store bytes (both item operands once) / both phases' time",
                                "achieved": 2 * op_b / (tot * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": 2 * op_b / (tot * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                "bytes_read_by_design": 3 * op_b})
    else:
        als, tt, a_mm, t_mm = o.hybrid_scores(rec.U, hu, uvec, rec.V_op, rec.iv_op)
        # one launch: user gather + bf16 conversion, both GEMMs, both rows'
        # min / max; bound by the two f32 score matrices it writes (+ the
        # bf16 item operands it reads)
        st = [("hybrid_scores (ALS + two-tower bf16 MFMA GEMMs, dk %d, + row min/max)" % rec.dk,
               lambda: o.hybrid_scores(rec.U, hu, uvec, rec.V_op, rec.iv_op),
               dict(bound="hbm", work=2 * 4.0 * B * N + 2 * 2.0 * rec.dk * N, peak=HBM_PEAK_GBS, unit="GB/s",
                    mfma_flops=2 * 2.0 * rec.dk * B * N))]
    if rec.precision == "exact":
        a_mm, t_mm = o.rows_minmax(als), o.rows_minmax(tt)
        st.append(("rows_minmax x2 (per-user min/max of both score rows)",
                   lambda: (o.rows_minmax(als), o.rows_minmax(tt)),
                   dict(bound="hbm", work=2 * 4.0 * B * N, peak=HBM_PEAK_GBS, unit="GB/s")))
    st += [("fuse_rows_topk (min-max fusion f64 + stable top-k)",
            lambda: o.fuse_rows_topk(als, tt, a_mm, t_mm, False, top_k, rec.offset),
            dict(bound="hbm", work=8.0 * B * N, peak=HBM_PEAK_GBS, unit="GB/s"))]
    out = []
    for name, fn, rf in st:
        fn()
        ms = ev_time(fn, reps, stream)
        r = roofline(rf["bound"], rf["work"], ms, rf["peak"], rf["unit"], name)
        if "mfma_flops" in rf:
            tf = rf["mfma_flops"] / (ms * 1e-3) / 1e12
            r["mfma_view"] = {"achieved": tf, "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                              "frac": tf / BF16_MFMA_PEAK_TFLOPS}
        out.append(r)
    dom = max(out, key=lambda r: r["avg_launch_ms"])
    return dict(dom, stages=out)


def cpu_baseline(eng, cfg, n_user_rows, n_item_rows, k=None):
    """C oracle on a bounded sample of the same matrix (rank 0, N=1)."""
    import numpy as np

    from oracle import build as obuild

    from oracle.cpu_baseline import cpu_model

    obuild.build()
    k = cfg["rank"] if k is None else int(k)

    def sample(csr, rows):
        ip = csr.indptr[: rows + 1].cpu().numpy()
        return ip, csr.indices[: int(ip[-1])].cpu().numpy(), csr.values[: int(ip[-1])].cpu().numpy()

    ucsr = sample(eng.user_csr, n_user_rows)
    icsc = sample(eng.item_csc, n_item_rows)
    U = eng.U[: cfg["users"], :k].cpu().numpy()
    V = eng.V[: cfg["items"], :k].cpu().numpy()
    t0 = time.perf_counter()
    obuild.half_sweep(*icsc, U, k, 0.1)
    t_item = time.perf_counter() - t0
    t0 = time.perf_counter()
    obuild.half_sweep(*ucsr, V, k, 0.1)
    t_user = time.perf_counter() - t0
    epoch_s = t_item * cfg["items"] / n_item_rows + t_user * cfg["users"] / n_user_rows
    return {
        "value": 1.0 / epoch_s, "unit": "epochs/s", "cores": int(obuild.load().oracle_max_threads()),
        "kind": "port", "cpu_model": cpu_model(),
        "sample": (f"C oracle (Spark 3.5.1 ALS restated: f64 dspr Gramian + dpptrf/dpptrs, OpenMP) on "
                   f"{n_item_rows} item rows + {n_user_rows} user rows of the same c2 matrix at rank {k}, "
                   f"{t_item + t_user:.1f} s measured, extrapolated to one full epoch"),
    }


def latest_profile():
    import glob

    c = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_prof_summary.json")))
    return c[-1] if c else None


def source_sha256(name):
    import hashlib

    with open(os.path.join(ROOT, "hybrid-als-twotower-recommender_amd", "csrc", name), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


# Counter evidence per bench line: the kernels a line's roofline is about
# (name prefixes in the profile's per-kernel table) and the source they come
# from; attached only when that source is the one profiled (sha256).
COUNTER_KERNELS = [
    ((), ["als_half_sweep_f64_kernel"], "als.hip"),
    (("scoring",), ["als_bound_filter_kernel", "als_rescore_topk_kernel", "als_prune_"], "score.hip"),
    (("hybrid_top5",), ["hx_"], "hybrid_exact.hip"),
    (("ingest",), ["sort_downsweep_kernel", "sort_upsweep_kernel", "mark_", "codes_", "descent_kernel"],
     "ingest.hip"),
    (("tt_item_vectors_c4",), ["tt_item_forward_mfma_kernel<8, 8, true, false, 16, true>"], "tt_mfma.hip"),
    (("tt_scoring_c4", "f32"), ["dot_res_kernel<false, 128, true"], "dot_topk.hip"),
    (("tt_scoring_c4", "bf16"), ["dot_res_kernel<true, 128, true"], "dot_topk.hip"),
    (("tt_scoring_c4", "f32_B1"), ["dot_gemv_kernel<128, true>"], "dot_gemv.hip"),
    (("tt_scoring_c4", "bf16_B1"), ["dot_res_kernel<true, 128, true"], "dot_topk.hip"),
    (("hybrid_top5_c5",), ["hyb_scores_kernel", "hp_", "dot_res_kernel<true, 256, true"], "hybrid_scores.hip"),
    (("tt_train",), ["tt_item_forward_mfma_kernel<4, 4, true, true", "tt_bwd_", "adam_sparse_group4_kernel"],
     "tt_mfma.hip"),
    (("api_hybrid_call", "cold_user"), ["cold_"], "cold_start.hip"),
    (("als_rank256",), ["als_half_sweep_wide_kernel"], "als_wide.hip"),
]


def attach_counters(line, pj, prof):
    """roofline["counters"] of every line: per kernel of the line the trace
    duration, the MFMA-busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over every
    SIMD's cycles), the effective clock and the HBM bytes per dispatch, from
    the newest profiles/r*_prof_summary.json when it profiled this tree's
    source of those kernels; otherwise null with the reason."""
    table = pj.get("kernels") if pj else None
    for path, prefixes, src in COUNTER_KERNELS:
        node = line
        for key in path:
            node = node.get(key) if isinstance(node, dict) else None
        if not isinstance(node, dict) or not isinstance(node.get("roofline"), dict):
            continue
        if not table:
            node["roofline"]["counters"] = None
            continue
        fresh = pj.get("sources_sha256", {}).get(src) == source_sha256(src)
        ks = {}
        if fresh:
            for name, e in sorted(table.items()):
                if any(name.startswith(p) for p in prefixes):
                    ks[name] = {k: e[k] for k in ("avg_ms", "mfma_busy_frac", "mfma_busy_by_grid", "eff_clock_GHz",
                                                  "hbm_bytes_per_dispatch_corrected") if k in e}
        node["roofline"]["counters"] = {
            "profile": os.path.relpath(prof, ROOT), "source": src, "source_matches_profile": fresh,
            "kernels": ks if fresh else None,
            "note": ("mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs), time-weighted "
                     "over the kernel's dispatches (mfma_busy_by_grid: per launch shape, e.g. the 1-user and the "
                     "1024-user c4 batches), reads low on dispatches < 0.3 ms; hbm bytes = FETCH_SIZE x 2 + "
                     "WRITE_SIZE (KiB, gfx950 16-B-load correction); separate PMC passes, scripts/gpu_profile.sh")}


def api_line(eng, n_users, n_items, k, reps, want_cpu):
    import contextlib
    import io

    import numpy as np
    import pandas as pd
    from sklearn.preprocessing import MinMaxScaler

    from src.als_model import ALSModel, DeviceALSFactors, DeviceSession
    from src.hybrid_system import HybridRecommendationSystem, fuse_device
    from src.two_tower_model import TwoTowerModel

    d = 64
    als = ALSModel(rank=k)
    als.spark = DeviceSession()
    als.model = DeviceALSFactors(np.arange(n_users), np.arange(n_items), eng.U[:n_users], eng.V[:n_items], k)
    # the two-tower user table also holds the cold users below (ids the ALS model never saw)
    tt = TwoTowerModel(n_users + 2048, n_items, 2651, 255, embedding_size=d, seed=4)
    tt.build_model()
    rng = np.random.default_rng(9)
    items = pd.DataFrame({"itemId": np.arange(n_items), "manufacturer_id": rng.integers(0, 2651, n_items),
                          "category_id": rng.integers(0, 255, n_items), "price": rng.random(n_items) * 100,
                          "average_review_rating": rng.integers(0, 19, n_items).astype(np.float64)})
    tt.scaler = MinMaxScaler().fit(items[["price", "average_review_rating"]])
    # the cold-start fallback's inputs (src/als_model.py:48,86): per-item content features + mean rating
    from src.data_preprocessing import get_item_features

    als.item_features = get_item_features(items)
    als.global_mean = items["average_review_rating"].mean()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    als._fallback()  # hrec_cold_fallback over every item (once per model)
    torch.cuda.synchronize()
    precompute_ms = (time.perf_counter() - t0) * 1e3
    h = HybridRecommendationSystem()
    h.als_model, h.twotower_model, h.models_loaded = als, tt, True
    ids = [int(i) for i in items["itemId"]]
    uids = [int(u) for u in rng.integers(0, n_users, reps + 1)]
    sink = io.StringIO()

    per_call = {}

    def timed(fn, key=None):
        fn(uids[0])
        torch.cuda.synchronize()
        ts = []
        t0 = time.perf_counter()
        for u in uids[1:]:
            c0 = time.perf_counter()
            fn(u)  # each call ends on the device -> host copy of its top-k (synchronous)
            ts.append(time.perf_counter() - c0)
        torch.cuda.synchronize()
        if key:
            per_call[key] = {"median_ms": float(np.median(ts)) * 1e3, "min_ms": float(np.min(ts)) * 1e3,
                             "max_ms": float(np.max(ts)) * 1e3}
        return (time.perf_counter() - t0) / reps * 1e3

    class Candidates:
        """all_items that both models score: iterates as a list of item ids
        (ALS side), indexes as the frame (two-tower side)."""

        def __iter__(self):
            return iter(ids)

        def __len__(self):
            return len(items)

        def __getitem__(self, key):
            return items[key]

    class IdArray(np.ndarray):
        """The same candidates as an integer id array (what the ALS side
        iterates, src/als_model.py:70, e.g. df["itemId"].unique() as the
        reference's tuning loop passes it, :155) that answers the two-tower
        side's column lookups (src/two_tower_model.py:138-143) from the frame."""

        def __getitem__(self, key):
            if isinstance(key, (str, list)):
                return items[key]
            return super().__getitem__(key)

    both = Candidates()
    arr = items["itemId"].to_numpy().view(IdArray)
    parts = {}
    with contextlib.redirect_stdout(sink):
        ref_ms = timed(lambda u: h.get_hybrid_recommendations(u, items, top_k=5), "reference_call")
        iter_ms = timed(lambda u: h.get_hybrid_recommendations(u, both, top_k=5), "api_call_iterable")
        arr_ms = timed(lambda u: h.get_hybrid_recommendations(u, arr, top_k=5), "api_call")
        top_api = h.get_hybrid_recommendations(uids[0], arr, top_k=5)
        top_iter = h.get_hybrid_recommendations(uids[0], both, top_k=5)
        parts["als.predict_for_user (id list)"] = timed(lambda u: als.predict_for_user(u, ids))
        parts["twotower.predict_for_user (item frame)"] = timed(lambda u: tt.predict_for_user(u, items))
        a, t = als.predict_for_user(uids[0], ids), tt.predict_for_user(uids[0], items)

        def fuse(_u):
            its, sa, st = h._union(a, t)
            _, idx, sc = fuse_device(sa, st, h.als_f1_score > h.twotower_f1_score, 5,
                                     scalers=(h.als_scaler, h.twotower_scaler))
            return [(its[i], np.float64(x)) for i, x in zip(idx, sc)]

        parts["_union + fuse_device top-5"] = timed(fuse)
        top = fuse(0)
        # cold users (the reference protocol's test users): ids the ALS model does not
        # know -> every ALS row takes the precomputed fallback, gathered on the device
        cold_uids = [n_users + 1000 + i for i in range(min(reps + 1, 1000))]
        cold_ms = timed(lambda u: h.get_hybrid_recommendations(cold_uids[u % len(cold_uids)], arr, top_k=5),
                        "cold_user_call")
        cu = cold_uids[0]
        top_cold = h.get_hybrid_recommendations(cu, arr, top_k=5)
        ca, ct = als.predict_for_user(cu, ids), tt.predict_for_user(cu, items)
        its, sa, st = h._union(ca, ct)
        _, cidx, csc = fuse_device(sa, st, h.als_f1_score > h.twotower_f1_score, 5)
        top_cold_list = [(its[i], np.float64(x)) for i, x in zip(cidx, csc)]
    work = sum(parts.values())

    # device share of one call: the same kernels on device-resident inputs
    # (ALS transform, item tower + user tower + Dot, fusion + top-6), HIP events
    stream = torch.cuda.current_stream()
    keys = np.arange(n_items, dtype=np.int64)
    dev_in = tt._device_inputs({"user_in": np.full(n_items, uids[0]), "item_id_in": keys,
                                "manufacturer_in": items["manufacturer_id"].values,
                                "category_in": items["category_id"].values,
                                "numeric_in": tt.scaler.transform(items[["price", "average_review_rating"]])})
    irows = als.model._lookup_device(keys)
    urow = torch.as_tensor(als.model._lookup(als.model.user_ids, [uids[0]]), device="cuda")

    def device_call():
        sa = _hrec.als_score(als.model.U, urow, als.model.Vt, irows, n_items, k)[0]
        uv = tt.model.user_vectors(dev_in[0][:1])
        iv = tt.model.item_vectors(*dev_in[1:])
        st = _hrec.tt_score(uv, iv).reshape(-1)
        return _hrec.fuse_topk(sa.double(), st, False, 6, want_fused=False)

    device_call()
    dev_ms = ev_time(device_call, reps, stream)
    item_bytes = n_items * (4.0 * k + 4.0 * d)  # each candidate's ALS factor row + tower vector, read once
    out = {"users_per_s": 1e3 / arr_ms, "pairs_per_s": n_items * 1e3 / arr_ms, "api_call_ms": arr_ms,
           "api_call_iterable_ms": iter_ms, "reference_call_ms": ref_ms, "per_call": per_call, "list_path_ms": work,
           "list_parts_ms": parts, "items": n_items, "top_k": 5, "reps": reps,
           "top5_nonempty": len(top_api) == 5,
           "api_top5_equals_list_path": [i for i, _ in top_api] == [i for i, _ in top] == [i for i, _ in top_iter],
           "roofline": {"kernel": "one call's device work (hrec_als_score + tt towers + hrec_tt_score + "
                                  "hrec_fuse_topk), HIP events", "bound": "hbm",
                        "achieved": item_bytes / (arr_ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": item_bytes / (arr_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                        "algorithmic_bytes": item_bytes,
                        "device_ms": dev_ms, "device_frac": item_bytes / (dev_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                        "host_share": max(0.0, 1.0 - dev_ms / arr_ms),
                        "note": ("algorithmic bytes = N (4k + 4d): every candidate's ALS item factor row and "
                                 "two-tower item vector read once; achieved over the whole API call (host "
                                 "work included: the share of the call that is not device time is host_share)")},
           "note": ("one user per call (the reference API, src/hybrid_system.py:95-116). api_call = "
                    "get_hybrid_recommendations(uid, candidates) with the candidates an integer id array that "
                    "also answers the two-tower side's column lookups (ALS reads it without a per-item Python "
                    "pass); api_call_iterable = the same candidates iterating as a Python list of ids; "
                    "reference_call = get_hybrid_recommendations(uid, item_frame) as the reference wires it "
                    "(ALS side -> [] by SURVEY D9). All run the array path (device scores -> device fusion + "
                    "top-6 -> tie check); list_path = the per-model predict_for_user lists + _union + "
                    "fuse_device (still taken on ties / duplicate ids / cold-start rows)")}
    cold_bytes = n_items * (4.0 * d + 8.0)  # each candidate's tower vector + its f64 fallback value, read once
    out["cold_user_call_ms"] = cold_ms
    out["cold_user"] = {
        "call_ms": cold_ms, "users_per_s": 1e3 / cold_ms, "fallback_precompute_ms": precompute_ms,
        "top5_nonempty": len(top_cold) == 5,
        "top5_equals_list_path": top_cold == top_cold_list,
        "roofline": {"kernel": "one cold call (fallback gather + tt towers + hrec_tt_score + hrec_fuse_topk), "
                               "whole API call", "bound": "hbm",
                     "achieved": cold_bytes / (cold_ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": cold_bytes / (cold_ms / 1e3) / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes": cold_bytes},
        "note": ("get_hybrid_recommendations(uid, id array) for user ids the ALS model does not know: every ALS "
                 "row is the precomputed cold-start fallback (hrec_cold_fallback once per model, "
                 "fallback_precompute_ms, over all items; src/als_model.py:78-86,93-104), gathered for the "
                 "candidates on the device; top5_equals_list_path compares with predict_for_user lists + "
                 "_union + fuse_device")}
    if want_cpu:
        from oracle import cpu_baseline as cb

        out["cpu_baseline"] = cb.api_call(n_items, k, d, 5)
        out["cold_user"]["cpu_baseline"] = cb.cold_call(n_items)
    return out



def c4_tower_check(tt4, it4, mn4, ct4, nu4, V4, n_rows=500):
    """BASELINE c4 at full size: 500 sampled rows of the 50M-item tower output
    against the f64 Keras graph (oracle/two_tower.py forward, rtol 1e-5 /
    atol 2e-5 as tests/test_gpu_api.py), on the host."""
    import numpy as np

    from oracle import two_tower as ott

    n = V4.shape[0]
    g = np.random.default_rng(77)
    rows = np.unique(np.concatenate([g.integers(0, n, n_rows), [0, n - 1]]))
    rt = torch.as_tensor(rows, device=V4.device)
    p = {name: t.detach().cpu().numpy() for name, t in tt4.tensors.items() if name not in ("user_emb", "item_emb")}
    p["item_emb"] = tt4.tensors["item_emb"].index_select(0, rt).cpu().numpy()
    p["user_emb"] = np.zeros((1, tt4.d), np.float32)
    ref = ott.forward(p, np.zeros(len(rows), np.int64), np.arange(len(rows)), mn4[rt].cpu().numpy(),
                      ct4[rt].cpu().numpy(), nu4[rt].cpu().numpy())["ivec"]
    got = V4.index_select(0, rt).cpu().numpy().astype(np.float64)
    err = np.abs(got - ref) - (1e-5 * np.abs(ref) + 2e-5)
    return {"rows_checked": int(len(rows)), "rows_match_oracle": bool(np.all(err <= 0)),
            "max_abs_err": float(np.max(np.abs(got - ref))),
            "tolerance": "|gpu - f64 graph| <= 1e-5 |ref| + 2e-5 (oracle/two_tower.py forward)"}


def c4_ranking_check(Ud, Vd, sc, k=5, chunk=1 << 20):
    """Top-k of 8 users over all items of the c4 catalogue vs the f64 ranking
    of the same operands (bf16: the bf16-rounded values), computed here in
    f64 chunks on the device; indices must agree wherever the f64 top-(k+1)
    is separated by more than the f32 score tolerance."""
    gi, gv = sc.topk(Ud, k)
    U64 = Ud.double()
    best_v, best_i = [], []
    for j0 in range(0, Vd.shape[0], chunk):
        s = U64 @ Vd[j0: j0 + chunk].double().T
        v, i = torch.topk(s, k + 1, dim=1, sorted=True)
        best_v.append(v)
        best_i.append(i + j0)
    v = torch.cat(best_v, 1)
    i = torch.cat(best_i, 1)
    # stable order: larger score first, ties -> smaller index
    key = torch.argsort(i, dim=1)
    v, i = v.gather(1, key), i.gather(1, key)
    order = torch.argsort(-v, dim=1, stable=True)[:, : k + 1]
    rv, ri = v.gather(1, order).cpu(), i.gather(1, order).cpu()
    gi = gi.cpu()
    checked, ok, tol = 0, True, 0.0
    for b in range(Ud.shape[0]):
        # f32 accumulation bound: 1e-6 x sum_c |u_c v_c| (tests/test_gpu_dot.py), x2 margin
        rows = Vd.index_select(0, ri[b].to(Vd.device)).double().abs()
        tol_b = 2e-6 * float((rows @ U64[b].abs()).max())
        tol = max(tol, tol_b)
        gaps = (rv[b, :-1] - rv[b, 1:]).tolist()
        if all(x > 2 * tol_b for x in gaps):
            checked += 1
            ok = ok and gi[b].tolist() == ri[b, :k].tolist()
    return {"users": int(Ud.shape[0]), "users_separated": checked, "top5_matches_f64_ranking": ok,
            "score_tol_max": tol, "rule": ("indices equal for every user whose f64 top-6 gaps all exceed 2 x tol_b, "
                                           "tol_b = 2e-6 x max sum_c |u_c v_c| over those items")}

def WANT_CPU(args, rank, world):
    """CPU baselines run on rank 0 at N = 1 only (a bounded sample each)."""
    return rank == 0 and world == 1 and not args.no_cpu_baseline


def launch_ranks(n):
    """--gpus N > 1 without a launcher (WORLD_SIZE unset): start N fresh rank
    processes through torch.distributed.run — before this process touches
    the GPU — and return their exit status. Each rank gets its own device
    (LOCAL_RANK) and RCCL; HREC_BENCH_BACKEND / HREC_BENCH_DEVICE pass
    through for the one-GPU gloo rehearsal."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd)


def max_over_ranks(x, world):
    t = torch.tensor([float(x)], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def run_als(cfg, world, rank, group, chunks, steps, warmup, accum_mode, stream):
    """One configuration's ALS fit timed: this rank's CSR / CSC shard
    generated on the device, `warmup` untimed + `steps` timed epochs (barrier
    + synchronize on both sides, max over ranks), then one compute-only epoch
    (the same kernels without the all-gathers) for the collective time that
    is not hidden. Returns (engine, csr, csc, facts)."""
    k = cfg["rank"]
    n_users, n_items = cfg["users"], cfg["items"]
    # ALS shards: chunk-interleaved when W > 1 so each chunk's all-gather
    # overlaps the next chunk's half-sweep. Parts balanced on cost = nnz + a
    # per-row solve term (RowLayout.balanced over every row's rating count)
    # when counting is cheap (the count is a hash over every (user, item)
    # pair: 1e11 at c2); at c3 (1e13 pairs, layout "equal") equal-count parts
    # of the uniform hash matrix, balanced in expectation (the nnz ratio is
    # reported)
    if world > 1 and cfg.get("layout") != "equal":
        u_lay = RowLayout.balanced(synthetic.row_counts(n_users, n_items, cfg["density"], False).cpu().numpy(),
                                   world, chunks)
        i_lay = RowLayout.balanced(synthetic.row_counts(n_users, n_items, cfg["density"], True).cpu().numpy(),
                                   world, 1)
        layout = "nnz-balanced contiguous parts"
    else:
        u_lay, i_lay = RowLayout.equal(n_users, world, chunks), RowLayout.equal(n_items, world, 1)
        layout = "equal-count contiguous parts" if world > 1 else "one shard"
    g0 = time.perf_counter()
    csr = synthetic.generate_layout(n_users, n_items, cfg["density"], False, u_lay, rank)
    csc = synthetic.generate_layout(n_users, n_items, cfg["density"], True, i_lay, rank)
    eng = DeviceALS(n_users, n_items, k, 0.1, csr, csc, world=world, rank=rank, group=group,
                    accum_mode=accum_mode, chunks=chunks, user_layout=u_lay, item_layout=i_lay)
    eng.init_user_factors(synthetic.SEED_INIT)
    torch.cuda.synchronize()
    gen_s = time.perf_counter() - g0

    nnz_local = torch.tensor([csr.nnz, csc.nnz], dtype=torch.int64, device="cuda")
    per_rank = torch.tensor([csr.nnz + csc.nnz], dtype=torch.int64, device="cuda")
    per_rank_nnz = [int(per_rank.item())]
    if world > 1:
        dist.all_reduce(nnz_local)
        allr = torch.zeros(world, dtype=torch.int64, device="cuda")
        dist.all_gather_into_tensor(allr, per_rank)
        per_rank_nnz = allr.tolist()
    nnz_user, nnz_item = (int(x) for x in nnz_local.tolist())

    for _ in range(warmup):
        eng.epoch()

    # Timed region: K epochs, barrier + synchronize on both sides.
    ev = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        # events on the launch stream; at W = 1 they bracket exactly the two
        # half-sweep kernels, at W > 1 also the all-gathers not hidden
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record(stream)
        eng.item_half_sweep()
        e[1].record(stream)
        eng.user_half_sweep()
        e[2].record(stream)
        ev.append(e)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    item_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / len(ev)
    user_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / len(ev)

    # the same epoch's kernels without the collectives (after the timed region)
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    c0.record(stream)
    eng.compute_only_epoch()
    c1.record(stream)
    torch.cuda.synchronize()
    compute_ms = max_over_ranks(c0.elapsed_time(c1), world)
    ms_per_step = elapsed / steps * 1e3
    facts = dict(k=k, n_users=n_users, n_items=n_items, elapsed=elapsed, ms_per_step=ms_per_step,
                 item_ms=item_ms, user_ms=user_ms, nnz_user=nnz_user, nnz_item=nnz_item, per_rank_nnz=per_rank_nnz,
                 layout=layout, gen_s=gen_s,
                 u0=u_lay.part_rows(rank)[0][0], u_per=csr.n_rows,
                 u_real=sum(c for _, c in u_lay.part_rows(rank)), i_real=sum(c for _, c in i_lay.part_rows(rank)),
                 collectives={"world_size": world, "epoch_ms": ms_per_step,
                              "compute_only_epoch_ms_max_over_ranks": compute_ms,
                              "collective_ms_not_hidden_per_epoch": max(0.0, ms_per_step - compute_ms),
                              "allgather_bytes_per_epoch_replicated": (eng.U.numel() + eng.V.numel()) * 4
                              if world > 1 else 0,
                              "note": ("epoch wall time (max over ranks) minus the same epoch's half-sweep "
                                       "kernels alone (one compute-only epoch, HIP events, max over ranks)")})
    return eng, csr, csc, facts


def c3_line(world, rank, group, chunks, epochs, stream):
    """The c3 sub-line: run_als on BASELINE configs[2] with `epochs` timed
    epochs (1 warmup), or the reason it was skipped (not enough free device
    memory on some rank for its CSR + CSC shard, decided on every rank)."""
    cfg = CONFIGS["c3"]
    k = cfg["rank"]
    nnz_rank = cfg["density"] * cfg["users"] * cfg["items"] / world
    need = 2 * nnz_rank * 8 * 1.02 + (cfg["users"] + cfg["items"]) * k * 4 * 3
    ok = torch.tensor([1 if torch.cuda.mem_get_info()[0] >= need else 0], dtype=torch.int64, device="cuda")
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if not int(ok.item()):
        return {"skipped": True, "reason": f"a rank has less than {need / 1e9:.0f} GB of free device memory "
                                           f"for its c3 shard (+ factors)"}
    e3, csr3, csc3, f = run_als(cfg, world, rank, group, chunks, epochs, 1, 0, stream)
    fl = algo_flops(csc3.nnz, f["i_real"], k) + algo_flops(csr3.nnz, f["u_real"], k)
    by = algo_bytes(csc3.nnz, f["i_real"], k) + algo_bytes(csr3.nnz, f["u_real"], k)
    ks = (f["item_ms"] + f["user_ms"]) / 1e3
    tf = fl / ks / 1e12
    tf_min = -max_over_ranks(-tf, world)  # the slowest rank's rate
    out = {"epochs_per_s": epochs / f["elapsed"], "ms_per_epoch": f["ms_per_step"], "epochs": epochs,
           "warmup": 1, "world_size": world, "rehearsal": bool(cfg.get("rehearsal")),
           "config": {"users": cfg["users"], "items": cfg["items"], "density": cfg["density"], "rank": k,
                      "nnz": f["nnz_user"], "nnz_check_csc": f["nnz_item"],
                      "shard_nnz_max_over_min": max(f["per_rank_nnz"]) / max(1, min(f["per_rank_nnz"])),
                      "shard_layout": f["layout"], "user_chunks_per_rank": chunks,
                      "generate_s": f["gen_s"]},
           "collectives": f["collectives"],
           "roofline": roofline("mfma", fl / 2, (f["item_ms"] + f["user_ms"]) / 2, F64_MFMA_PEAK_TFLOPS, "TFLOP/s",
                                "als_half_sweep_f64_kernel (item + user launches, rank 0's shard)",
                                slowest_rank_TFLOPs=tf_min,
                                kernel_ms_per_epoch={"item": f["item_ms"], "user": f["user_ms"]},
                                gather_view={"algorithmic_GBps": by / ks / 1e9, "hbm_peak_GBps": HBM_PEAK_GBS,
                                             "frac": by / ks / 1e9 / HBM_PEAK_GBS}),
           "north_star": {"target_epochs_per_s": 50, "note": (
               "the exact f64-accumulated ALS flops of one c3 epoch (1.07e14 per GPU) bound 8 MI355X at "
               "~0.73 epochs/s on the f64 matrix cores (DESIGN §5); the rate here is that bound's fraction")}}
    del e3, csr3, csc3
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--score-users", type=int, default=1024)
    ap.add_argument("--hybrid-users", type=int, default=256,
                    help="users per batch of the end-to-end hybrid top-5 measurement (0 = skip)")
    ap.add_argument("--c4-items", type=int, default=50_000_000,
                    help="two-tower scoring (c4): candidate items in total over all ranks (0 = skip)")
    ap.add_argument("--c4-users", type=int, default=1024)
    ap.add_argument("--c5-users", type=int, default=None,
                    help="users per batch of the c5 hybrid top-5 (rank 256 + d 256, bf16; 0 = skip; "
                         "default 256, 0 with --config c3)")
    ap.add_argument("--cpu-user-rows", type=int, default=600000)
    ap.add_argument("--cpu-item-rows", type=int, default=60000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-score-users", type=int, default=1024,
                    help="users of the scoring batch timed by the C JVM-exact scoring baseline")
    ap.add_argument("--rank256-epochs", type=int, default=None,
                    help="timed rank-256 ALS epochs on the same matrix (BASELINE c5's ALS half; 0 = skip; "
                         "default 1, 0 with --config c3)")
    ap.add_argument("--c3-epochs", type=int, default=None,
                    help="timed epochs of the c3 sub-line (BASELINE configs[2]: 10M x 1M, 1 %%, rank 64, "
                         "8 GPUs), run after the c2 lines when 8 or more ranks are present; default 2")
    ap.add_argument("--api-reps", type=int, default=50,
                    help="users timed through HybridRecommendationSystem.get_hybrid_recommendations (0 = skip)")
    ap.add_argument("--chunks", type=int, default=4,
                    help="W > 1: user-side ALS row chunks per rank (per-chunk all-gathers overlap the next chunk)")
    ap.add_argument("--tt-steps", type=int, default=50,
                    help="two-tower training steps timed (c2 tables, d = 64, batch 256; 0 = skip)")
    ap.add_argument("--no-ingest", dest="ingest", action="store_false",
                    help="skip the COO -> CSR/CSC ingest measurement")
    ap.add_argument("--traffic-json", default=None,
                    help="rocprofv3 PMC summary (scripts/gpu_profile.sh) for roofline.traffic "
                         "(default: the newest profiles/r*_prof_summary.json)")
    ap.add_argument("--accum-mode", type=int, default=0, choices=[0, 1],
                    help="0: f64 matrix-core Gramian; 1: f32 matrix cores, f64 across 16-rating chunks")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    cfg = CONFIGS[args.config]
    if world < cfg.get("min_world", 1):
        raise SystemExit(f"--config {args.config} ({cfg['users']} x {cfg['items']}, density {cfg['density']}) is "
                         f"BASELINE's {cfg['min_world']}-GPU configuration: one rank's share is sized for "
                         f"{cfg['min_world']} ranks (one GPU each); run it with --gpus {cfg['min_world']}, "
                         f"got {world}")
    big = args.config == "c3"
    if args.c5_users is None:
        args.c5_users = 0 if big else 256
    if args.rank256_epochs is None:
        args.rank256_epochs = 0 if big else 1
    if args.c3_epochs is None:
        args.c3_epochs = 2
    # HREC_BENCH_BACKEND=gloo + HREC_BENCH_DEVICE=0: rehearsal of the W > 1
    # flow with every rank on one GPU (RCCL refuses two ranks per device);
    # the driver's multi-GPU runs use the defaults (RCCL, one GPU per rank).
    backend = os.environ.get("HREC_BENCH_BACKEND", "nccl")
    dev = int(os.environ.get("HREC_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(dev)
    group = None
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        group = dist.group.WORLD

    stream = torch.cuda.current_stream()
    chunks = args.chunks if world > 1 else 1
    eng, csr, csc, als = run_als(cfg, world, rank, group, chunks, args.steps, args.warmup, args.accum_mode, stream)
    k, n_users, n_items = als["k"], als["n_users"], als["n_items"]
    u0, u_per = als["u0"], als["u_per"]
    u_real, i_real = als["u_real"], als["i_real"]
    item_ms, user_ms, elapsed = als["item_ms"], als["user_ms"], als["elapsed"]
    nnz_user, nnz_item, per_rank_nnz = als["nnz_user"], als["nnz_item"], als["per_rank_nnz"]
    # per-rank algorithmic work of one epoch (both launches of the kernel; the
    # rank's real rows, its layout padding excluded)
    flops = algo_flops(csc.nnz, i_real, k) + algo_flops(csr.nnz, u_real, k)
    bytes_ = algo_bytes(csc.nnz, i_real, k) + algo_bytes(csr.nnz, u_real, k)
    # item shards of the scoring / hybrid lines (equal contiguous ranges)
    i0, i_per = shard_range(n_items, world, rank)
    kern_s = (item_ms + user_ms) / 1e3
    achieved_tf = flops / kern_s / 1e12

    # Scoring: B users x all items, JVM-exact dot consumed by a stable top-5
    # (hrec_als_score_topk_pruned: bf16 matrix-core bound, the JVM chain only
    # for the pairs it keeps; the score matrix is never written). The fused
    # path (hrec_als_score_topk: the chain over every pair) is timed beside it
    # and must return the same bits.
    scoring = None
    if rank == 0 and args.score_users > 0:
        Vrow = eng.item_factor_rows(0, n_items).contiguous()
        Vt = _hrec.transpose(Vrow)
        ops = _hrec.als_items_bf16(Vrow, k)  # once per item matrix
        B = args.score_users
        users = eng.user_rows(torch.arange(B, dtype=torch.int64, device="cuda") * (n_users // B))
        ws = torch.empty(int(_hrec.lib().hrec_als_score_topk_pruned_workspace_bytes(B, n_items, 5, k)),
                         dtype=torch.uint8, device="cuda")

        def pruned():
            return _hrec.als_score_topk_pruned(eng.U, users, Vt, Vrow, ops, n_items, k, 5, workspace=ws)

        def fused():
            return _hrec.als_score_topk(eng.U, users, Vt, n_items, k, 5)

        def clock(fn, reps):
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            s0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - s0) / reps

        sc_s = clock(pruned, 20)
        fu_s = clock(fused, 5)
        (pi, pv), (fi, fv) = pruned(), fused()
        same = bool(torch.equal(pi, fi) and torch.equal(pv.view(torch.int32), fv.view(torch.int32)))
        kept = _hrec.als_topk_pruned_counts(ws, B, n_items, 5, k)
        dk = 32 if k <= 32 else (64 if k <= 64 else (128 if k <= 128 else 256))
        pps = B * n_items / sc_s
        scoring = {"pairs_per_s": pps, "ms_per_batch": sc_s * 1e3, "users": B,
                   "items": n_items, "top_k": 5, "dtype": "f32 (JVM-exact, no FMA) behind a bf16 bound",
                   "kernel": "hrec_als_score_topk_pruned (bf16 wave-tile maxima of 32768 items -> a sample bound; "
                             "bf16 matrix-core bound filter over every pair; JVM-exact chain over the kept pairs + "
                             "stable top-k in one block per user; an overflow resolved on the device by the gated "
                             "exact top-k, so a call needs no host read)",
                   "fused_ms_per_batch": fu_s * 1e3, "fused_pairs_per_s": B * n_items / fu_s,
                   "pruned_equals_fused": same,
                   "pairs_per_user": {"bound_kept_mean": float(kept[0].float().mean()),
                                      "bound_kept_max": int(kept[0].max()),
                                      "survivors_mean": float(kept[1].float().mean()),
                                      "survivors_max": int(kept[1].max())},
                   # every pair passes through the bf16 bound GEMM (2 dk flops per pair on
                   # the matrix cores); the exact chain runs on the kept pairs only
                   "roofline": {"bound": "mfma-bf16 (the bound pass over every pair)",
                                "achieved": pps * 2 * dk / 1e12, "peak": BF16_MFMA_PEAK_TFLOPS,
                                "unit": "TFLOP/s", "frac": pps * 2 * dk / 1e12 / BF16_MFMA_PEAK_TFLOPS,
                                "fused_valu_frac": B * n_items / fu_s * 2 * k / 1e12 / F32_VALU_MULADD_TFLOPS,
                                "note": "achieved over the whole call (sample bound, bound filter, exact "
                                        "chain, top-k); fused_valu_frac: the fused path against the f32 "
                                        "mul+add VALU rate its chain over every pair is bound by"}}
        if world == 1 and not args.no_cpu_baseline:
            from oracle import cpu_baseline as cb

            su = users[: args.cpu_score_users].cpu().numpy()
            scoring["cpu_baseline"] = cb.als_scoring(eng.U[su].cpu().numpy(), eng.item_factor_rows(0, n_items).cpu().numpy(),
                                                     k, 5, B)

    # End-to-end hybrid top-5 (HybridRecommendationSystem.get_hybrid_recommendations
    # for a batch of users): JVM-exact ALS scores + two-tower Dot (d=64, Keras
    # init) + per-model min-max fusion + stable top-5, items sharded across
    # ranks with RCCL all-reduce (min/max) and all-gather (candidates).
    hybrid = None
    if args.hybrid_users > 0:
        d = 64
        n_loc = max(0, min(i_per, n_items - i0))
        tt = DeviceTwoTower(n_users, n_items, 2651, 255, d, seed=1)
        g = torch.Generator().manual_seed(5)
        items = torch.arange(i0, i0 + n_loc, dtype=torch.int32)
        man = torch.randint(0, 2651, (n_items,), generator=g, dtype=torch.int32)[i0: i0 + n_loc]
        cat = torch.randint(0, 255, (n_items,), generator=g, dtype=torch.int32)[i0: i0 + n_loc]
        num = torch.rand((n_items, 2), generator=g)[i0: i0 + n_loc].contiguous()
        ivec = tt.item_vectors(items.cuda(), man.cuda(), cat.cuda(), num.cuda())
        Vt_loc = _hrec.transpose(eng.item_factor_rows(i0, n_loc).contiguous())
        rec = ShardedRecommender(eng.U, Vt_loc, ivec, i0, k, world=world, rank=rank, group=group)
        Bh = args.hybrid_users
        hu_ids = (torch.arange(Bh, dtype=torch.int64) * (n_users // Bh)).cuda()
        hu = eng.user_rows(hu_ids)  # rows of the (layout-ordered) user factor buffer
        uvec = tt.user_vectors(hu_ids.to(torch.int32))
        hs_g, hs_eager = time_recommend(rec, hu, uvec, world)
        hs, how = recommend_line_timing(hs_g, hs_eager)
        hybrid = {"pairs_per_s": Bh * n_items / hs, "ms_per_batch": hs * 1e3, "users": Bh, "items": n_items,
                  "eager_ms_per_batch": (hs_eager if hs_eager else hs_g) * 1e3,
                  "graph_ms_per_batch": hs_g * 1e3 if hs_eager else None, "launch": how,
                  "top_k": 5, "d": d, "items_sharded_over": world,
                  "steps": ("exact pruned hybrid (hrec_hybrid_exact_*: split-bf16 bound GEMMs of both models, "
                            "no score matrices; the candidate groups rescored by the JVM-exact ALS chain and the f32 "
                            "MFMA Dot; min-max fusion f64 + stable top-5, bit for bit the materialised path)"
                            if getattr(rec, "pruned_exact", False) else
                            "ALS JVM-exact f32 + two-tower f32 MFMA Dot + min-max fusion f64 + stable top-5")}
        if world == 1:
            hybrid["roofline"] = hybrid_stages(rec, hu, uvec, 5, 10, stream)
        if WANT_CPU(args, rank, world):
            from oracle import cpu_baseline as cb

            hybrid["cpu_baseline"] = cb.hybrid(Bh, n_items, k, d, 5)
        del rec, tt

    # BASELINE c5: rank-256 ALS factors + d = 256 two-tower vectors in bf16,
    # end-to-end hybrid top-5 over c2's items (sharded): both score matrices
    # on the bf16 matrix cores, per-model min-max fusion, stable top-5, C2/C3.
    # Factors are Spark-style random init (hrec_als_init_factors) — throughput
    # does not depend on their values; the rank-256 half-sweep is measured
    # separately (scripts/wide_quick.py).
    hybrid_c5 = None
    if args.c5_users > 0:
        k5, d5 = 256, 256
        n_loc = max(0, min(i_per, n_items - i0))
        U5 = torch.zeros((n_users, k5), dtype=torch.float32, device="cuda")
        _hrec.als_init_factors(synthetic.SEED_INIT, 0, n_users, k5, k5, U5)
        V5 = torch.zeros((n_loc, k5), dtype=torch.float32, device="cuda")
        _hrec.als_init_factors(synthetic.SEED_INIT + 1, i0, n_loc, k5, k5, V5)
        tt5 = DeviceTwoTower(n_users, n_items, 2651, 255, d5, seed=2)
        g5 = torch.Generator().manual_seed(6)
        items5 = torch.arange(i0, i0 + n_loc, dtype=torch.int32)
        man5 = torch.randint(0, 2651, (n_items,), generator=g5, dtype=torch.int32)[i0: i0 + n_loc]
        cat5 = torch.randint(0, 255, (n_items,), generator=g5, dtype=torch.int32)[i0: i0 + n_loc]
        num5 = torch.rand((n_items, 2), generator=g5)[i0: i0 + n_loc].contiguous()
        iv5 = tt5.item_vectors(items5.cuda(), man5.cuda(), cat5.cuda(), num5.cuda())
        rec5 = ShardedRecommender(U5, None, iv5, i0, k5, world=world, rank=rank, group=group,
                                  precision="bf16", V_local=V5)
        B5 = args.c5_users
        hu5 = (torch.arange(B5, dtype=torch.int64) * (n_users // B5)).cuda()
        uv5 = tt5.user_vectors(hu5.to(torch.int32))
        hs_g, hs_eager = time_recommend(rec5, hu5, uv5, world)
        hs, how = recommend_line_timing(hs_g, hs_eager)
        hybrid_c5 = {"pairs_per_s": B5 * n_items / hs, "ms_per_batch": hs * 1e3, "users": B5, "items": n_items,
                     "eager_ms_per_batch": (hs_eager if hs_eager else hs_g) * 1e3,
                     "graph_ms_per_batch": hs_g * 1e3 if hs_eager else None, "launch": how,
                     "top_k": 5, "rank": k5, "d": d5, "dtype": "bf16 operands, f32 accumulation",
                     "items_sharded_over": world,
                     "steps": ("pruned bf16 hybrid (hrec_hybrid_prune_minmax: both GEMMs, row min/max, no score "
                               "stores; hrec_hybrid_prune_topk: bound from the group maxima + the heavier model's "
                               "GEMM with a survivor filter + the survivors' light scores and fusion + stable "
                               "top-5; exact unfused fallback gated on the device)")}
        if world == 1:
            hybrid_c5["roofline"] = hybrid_stages(rec5, hu5, uv5, 5, 10, stream)
        if WANT_CPU(args, rank, world):
            from oracle import cpu_baseline as cb

            hybrid_c5["cpu_baseline"] = cb.hybrid(B5, n_items, k5, d5, 5)
        del U5, V5, tt5, rec5, iv5
        torch.cuda.empty_cache()

    # BASELINE c5's ALS half: rank 256 on c2's matrix (K1w,
    # als_half_sweep_wide_kernel, one 8-wave workgroup per row), same shards
    # and all-gathers as the headline; one untimed + E timed epochs.
    als256 = None
    if args.rank256_epochs > 0:
        k256 = 256
        e256 = DeviceALS(n_users, n_items, k256, 0.1, csr, csc, world=world, rank=rank, group=group, chunks=chunks,
                         user_layout=eng.u_layout, item_layout=eng.i_layout)
        e256.init_user_factors(synthetic.SEED_INIT)
        e256.epoch()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ev256 = []
        w0 = time.perf_counter()
        for _ in range(args.rank256_epochs):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(stream)
            e256.item_half_sweep()
            e[1].record(stream)
            e256.user_half_sweep()
            e[2].record(stream)
            ev256.append(e)
        torch.cuda.synchronize()
        wt = torch.tensor([(time.perf_counter() - w0) / args.rank256_epochs], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(wt, op=dist.ReduceOp.MAX)
        it_ms = sum(e[0].elapsed_time(e[1]) for e in ev256) / len(ev256)
        ut_ms = sum(e[1].elapsed_time(e[2]) for e in ev256) / len(ev256)
        fl256 = algo_flops(csc.nnz, i_real, k256) + algo_flops(csr.nnz, u_real, k256)
        als256 = {"epochs_per_s": 1.0 / float(wt.item()), "ms_per_epoch": float(wt.item()) * 1e3, "rank": k256,
                  "epochs": args.rank256_epochs, "kernel_ms_per_epoch": {"item": it_ms, "user": ut_ms},
                  "roofline": roofline("mfma", fl256 / 2, (it_ms + ut_ms) / 2, F64_MFMA_PEAK_TFLOPS, "TFLOP/s",
                                       "als_half_sweep_wide_kernel (item + user launches)")}
        if WANT_CPU(args, rank, world):
            # ~16x the per-rating Gramian work of rank 64: a 16x smaller row sample
            als256["cpu_baseline"] = cpu_baseline(e256, cfg, max(args.cpu_user_rows // 16, 1),
                                                  max(args.cpu_item_rows // 16, 1), k=k256)
        del e256
        torch.cuda.empty_cache()

    # The drop-in API call itself: HybridRecommendationSystem.
    # get_hybrid_recommendations for ONE user over c2's 100k candidate items,
    # models in memory (ALS factors of this run, a d = 64 two-tower on c2's
    # tables). The reference hands the same `all_items` object to both models
    # (src/hybrid_system.py:100-101): with the item DataFrame the ALS side
    # fails as the reference's does -> "reference_call"; the
    # "api_call" hands both models candidates they can score (ids for ALS,
    # the frame for the two-tower side). Both take the array path (device
    # scores -> device fusion + top-6 -> tie check); "list_path" times the
    # per-model predict_for_user lists + _union + fuse_device it replaces.
    api = None
    if rank == 0 and world == 1 and args.api_reps > 0:
        api = api_line(eng, n_users, n_items, k, args.api_reps, WANT_CPU(args, rank, world))

    # Ingest (§8(f) row 1, ALSModel.train's DataFrame -> CSR/CSC step): the
    # rank's user shard as COO columns (int64 ids, ratings) -> id codes +
    # CSR + CSC on the device (hrec_encode_ids x2, hrec_coo_to_csr x2).
    ingest = None
    if world == 1 and args.ingest:
        counts = csr.indptr[1:] - csr.indptr[:-1]
        uid = torch.repeat_interleave(torch.arange(u0, u0 + u_per, dtype=torch.int64, device="cuda"), counts)
        iid = csr.indices.to(torch.int64)
        vals = csr.values

        def run_ingest():
            _, urow, u_ord, u_ptr = _hrec.encode_ids(uid, (u0, u0 + u_per - 1), order=True)
            iu, irow, i_ord, _ = _hrec.encode_ids(iid, (0, n_items - 1), order=True)
            # grouped by user: the codes are the CSR (its order read by the marking pass)
            a = _hrec.coo_to_csr(urow, irow, vals, u_per, alias=True, rows_in_order=u_ord, indptr=u_ptr)
            b = _hrec.coo_to_csr(irow, urow, vals, int(iu.numel()), rows_in_order=i_ord)
            return a, b

        run_ingest()
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        out = run_ingest()
        torch.cuda.synchronize()
        gs = time.perf_counter() - g0
        ok = bool(torch.equal(out[0][0], csr.indptr) and torch.equal(out[0][1], csr.indices))
        ingest = {"ratings_per_s": csr.nnz / gs, "ms": gs * 1e3, "ratings": csr.nnz,
                  "steps": ("encode user ids + encode item ids (presence table / bitmap + rank; the ids' order "
                            "read by the marking pass) + CSR (rows grouped by user: the item codes and ratings ARE "
                            "the CSR, indptr from the row codes) + CSC (2-pass stable radix sort, 10240-entry "
                            "tiles, each row's start by atomicMin in the last pass)"),
                  "csr_matches_generator": ok,
                  # algorithmic bytes per rating: read user id, item id (int64) + rating (f32) = 20 B; write
                  # both id codes (2 x int32) + the CSC column/value arrays (int32 + f32) = 16 B (the CSR's
                  # arrays are the item codes and the ratings themselves)
                  "roofline": roofline("hbm", 36.0 * csr.nnz, gs * 1e3, HBM_PEAK_GBS, "GB/s",
                                       "ingest (4 launches' sequence: encode_ids x2 + coo_to_csr x2, wall clock)",
                                       note=("two radix passes for the CSC: the bytes moved are a multiple "
                                             "of the algorithmic 36 B per rating (44 B before round 5 counted "
                                             "the CSR copy)"))}
        if WANT_CPU(args, rank, world):
            import numpy as np

            from oracle.cpu_baseline import cpu_model

            S = min(int(csr.nnz), 20_000_000)
            hu, hi, hv = uid[:S].cpu().numpy(), iid[:S].cpu().numpy(), vals[:S].cpu().numpy()
            c0 = time.perf_counter()
            _, hur = np.unique(hu, return_inverse=True)
            ius, hir = np.unique(hi, return_inverse=True)
            o1 = np.argsort(hur, kind="stable")
            o2 = np.argsort(hir, kind="stable")
            _ = (hir[o1], hv[o1], hur[o2], hv[o2], np.bincount(hur), np.bincount(hir))
            cs = time.perf_counter() - c0
            ingest["cpu_baseline"] = {
                "value": S / cs, "unit": "ratings/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
                "sample": (f"numpy (the reference's ALSModel.train path is a Spark DataFrame; restated as "
                           f"np.unique(return_inverse) x2 + stable argsort CSR/CSC) on the first {S} of the "
                           f"{csr.nnz} ratings, {cs:.1f} s")}
        del uid, iid, out
        torch.cuda.empty_cache()

    # Two-tower scoring at BASELINE c4: d = 128, 50M candidate items, items
    # sharded over the ranks. First the catalogue's item vectors are
    # precomputed by the item tower (Keras graph, src/two_tower_model.py:38-66,
    # K4m on the f32 matrix cores; random Keras init of a 50M-row item table,
    # c2's 2651 manufacturers / 255 categories) — its own line,
    # tt_item_vectors_c4; then one batch of user-tower vectors is ranked
    # top-5 against every item (fused dot + filter + top-k; the [B, N] score
    # matrix is never written), C3 merge across ranks.
    tt_c4, tt_iv = None, None
    if args.c4_items > 0:
        tt_c4 = {}
        d4 = 128
        c0, c_per = shard_range(args.c4_items, world, rank)
        c_loc = max(0, min(c_per, args.c4_items - c0))
        tt4 = DeviceTwoTower(args.c4_users, c_loc, 2651, 255, d4, seed=1000 + rank, device_init=True)
        g4 = torch.Generator(device="cuda").manual_seed(2000 + rank)
        it4 = torch.arange(c_loc, dtype=torch.int32, device="cuda")
        mn4 = torch.randint(0, 2651, (c_loc,), device="cuda", generator=g4, dtype=torch.int32)
        ct4 = torch.randint(0, 255, (c_loc,), device="cuda", generator=g4, dtype=torch.int32)
        nu4 = torch.rand((c_loc, 2), device="cuda", generator=g4)
        V4 = tt4.item_vectors(it4, mn4, ct4, nu4)  # warm
        torch.cuda.synchronize()
        reps4 = 3
        q0 = time.perf_counter()
        iv_ms = ev_time(lambda: tt4.item_vectors(it4, mn4, ct4, nu4, out=V4), reps4, stream)
        it_t = torch.tensor([(time.perf_counter() - q0) / reps4], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(it_t, op=dist.ReduceOp.MAX)
        iv_bytes = c_loc * (4 * d4 + 64 + 8 + 12 + 4 * d4)
        tt_iv = {"items_per_s": args.c4_items / float(it_t.item()), "ms": float(it_t.item()) * 1e3,
                 "items": args.c4_items, "d": d4, "items_sharded_over": world,
                 "kernel": "tt_item_forward_mfma_kernel (Dense(16, relu) + concat + Dense(d) on f32 MFMA + LN)",
                 "roofline": roofline("mfma", 2.0 * (d4 + 32) * d4 * c_loc, iv_ms, F32_MFMA_PEAK_TFLOPS, "TFLOP/s",
                                      "tt_item_forward_mfma_kernel",
                                      hbm_view={"algorithmic_bytes": iv_bytes,
                                                "GBps": iv_bytes / (iv_ms / 1e3) / 1e9,
                                                "frac": iv_bytes / (iv_ms / 1e3) / 1e9 / HBM_PEAK_GBS})}
        if WANT_CPU(args, rank, world):
            from oracle import cpu_baseline as cb

            tt_iv["cpu_baseline"] = cb.item_vectors(args.c4_items // 100, args.c4_items, d4)
        U4 = tt4.user_vectors(torch.arange(args.c4_users, dtype=torch.int32, device="cuda"))
        if world == 1:
            tt_c4["tower_check"] = c4_tower_check(tt4, it4, mn4, ct4, nu4, V4)
        del tt4, it4, mn4, ct4, nu4
        torch.cuda.empty_cache()
        for name, dt, peak in (("f32", torch.float32, F32_MFMA_PEAK_TFLOPS),
                               ("bf16", torch.bfloat16, BF16_MFMA_PEAK_TFLOPS)):
            Vd = _hrec.dot_operand(V4, dt)
            Ud = _hrec.dot_operand(U4, dt)
            sc = ShardedScorer(Vd, c0, world=world, rank=rank, group=group)
            for nb in (args.c4_users, 1):  # B in {1, 1024}
                Ub = Ud[:nb].contiguous()
                sc.topk(Ub, 5)
                if world > 1:
                    dist.barrier()
                torch.cuda.synchronize()
                reps = 3 if nb > 1 else 10
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                q0 = time.perf_counter()
                e0.record(stream)
                for _ in range(reps):
                    sc.topk(Ub, 5)
                e1.record(stream)
                torch.cuda.synchronize()
                qt = torch.tensor([(time.perf_counter() - q0) / reps], dtype=torch.float64, device="cuda")
                if world > 1:
                    dist.all_reduce(qt, op=dist.ReduceOp.MAX)
                qs = float(qt.item())
                local_s = e0.elapsed_time(e1) / reps / 1e3  # this rank's launches, HIP events on the launch stream
                if nb > 1:
                    tf = 2.0 * nb * c_loc * d4 / local_s / 1e12
                    tt_c4[name] = {"pairs_per_s": nb * args.c4_items / qs, "ms_per_batch": qs * 1e3,
                                   "roofline": {"bound": "mfma", "achieved": tf, "peak": peak, "unit": "TFLOP/s",
                                                "frac": tf / peak}}
                else:
                    # one user: a GEMV, bound by reading every item operand once
                    ib = float(c_loc) * Vd.shape[1] * Vd.element_size()
                    gbs = ib / local_s / 1e9
                    tt_c4[name + "_B1"] = {"pairs_per_s": args.c4_items / qs, "ms_per_batch": qs * 1e3, "users": 1,
                                           "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS,
                                                        "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                                                        "algorithmic_bytes": ib,
                                                        "note": "item operand bytes of this rank read once "
                                                                "(N x dk x element size) / HIP-event time"}}
            if world == 1:
                tt_c4[name]["ranking_check"] = c4_ranking_check(Ud[:8].contiguous(), Vd, sc)
            del Vd, Ud
        if WANT_CPU(args, rank, world):
            from oracle import cpu_baseline as cb

            tt_c4["cpu_baseline"] = cb.tt_scoring(args.c4_items // 100, args.c4_items, args.c4_users, d4, 5)
        tt_c4.update({"users": args.c4_users, "items": args.c4_items, "d": d4, "top_k": 5,
                      "items_sharded_over": world,
                      "kernel": "hrec_dot_topk (sample bound + fused matrix-core dot + survivor filter + exact top-k)"})
        del V4, U4
        torch.cuda.empty_cache()

    # Two-tower training (Keras fit step, src/two_tower_model.py:111): c2's
    # tables at d = 64 (1M users, 100k items, 2651 manufacturers, 255
    # categories), batch 256, one step = forward + MSE + backward + Keras-exact
    # Adam. Keras' sparse Adam decays m and v of the WHOLE table every step
    # [ext: optimizer_v2/adam.py], so a step is bound by that HBM sweep:
    # 6 x 4 B (var, m, v read + write) per table element. W > 1 trains
    # replicas (sharding would change Keras' batch semantics): rank 0 only.
    tt_train = None
    if rank == 0 and world == 1 and args.tt_steps > 0:
        dtt = 64
        n_man, n_cat = 2651, 255
        tt = DeviceTwoTower(n_users, n_items, n_man, n_cat, dtt, seed=3)
        Bt = 256
        gt = torch.Generator(device="cuda").manual_seed(11)
        nb = 16  # distinct pre-generated batches, cycled
        bu = torch.randint(0, n_users, (nb, Bt), device="cuda", generator=gt, dtype=torch.int32)
        bi = torch.randint(0, n_items, (nb, Bt), device="cuda", generator=gt, dtype=torch.int32)
        bm = torch.randint(0, n_man, (nb, Bt), device="cuda", generator=gt, dtype=torch.int32)
        bc = torch.randint(0, n_cat, (nb, Bt), device="cuda", generator=gt, dtype=torch.int32)
        bx = torch.rand((nb, Bt, 2), device="cuda", generator=gt)
        by = torch.randint(0, 19, (nb, Bt), device="cuda", generator=gt).to(torch.float32)
        for j in range(3):
            tt.train_step(bu[j], bi[j], bm[j], bc[j], bx[j], by[j])
        torch.cuda.synchronize()
        te0, te1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0t = time.perf_counter()
        te0.record(stream)
        for j in range(args.tt_steps):
            q = j % nb
            tt.train_step(bu[q], bi[q], bm[q], bc[q], bx[q], by[q])
        te1.record(stream)
        torch.cuda.synchronize()
        tts = (time.perf_counter() - t0t) / args.tt_steps
        dev_s = te0.elapsed_time(te1) / args.tt_steps / 1e3
        tab_elems = n_users * dtt + n_items * dtt + (n_man + n_cat) * 8
        step_bytes = 6 * 4 * (tab_elems + tt.n_dense)
        tt_train = {"samples_per_s": Bt / tts, "ms_per_step": tts * 1e3, "batch": Bt, "d": dtt,
                    "tables": {"users": n_users, "items": n_items, "manufacturers": n_man, "categories": n_cat},
                    "steps": args.tt_steps,
                    "step": ("hrec_tt_forward_backward + hrec_adam_dense + Keras-exact sparse Adam on 4 tables "
                             + ("(hrec_adam_sparse_tables_phase: untouched-rows sweep on a side stream beside the "
                                "forward / backward)" if tt._phased else "(hrec_adam_sparse_tables, one stream)")),
                    "roofline": {"bound": "hbm", "achieved": step_bytes / dev_s / 1e9, "peak": HBM_PEAK_GBS,
                                 "unit": "GB/s", "frac": step_bytes / dev_s / 1e9 / HBM_PEAK_GBS,
                                 "algorithmic_bytes_per_step": step_bytes}}
        del tt, bu, bi, bm, bc, bx, by
        if not args.no_cpu_baseline:
            from oracle import cpu_baseline as cb

            tt_train["cpu_baseline"] = cb.tt_train(n_users, n_items, n_man, n_cat, dtt, Bt, 5)
        torch.cuda.empty_cache()

    # roofline.traffic: PMC bytes per launch from the newest committed
    # rocprofv3 summary (scripts/gpu_profile.sh), used only when the kernel
    # source it profiled is the one this tree runs (sha256 stamped by
    # scripts/summarize_profile.py); otherwise null + the reason.
    traffic, traffic_src, tsw, pj, fresh = None, None, None, {}, {}
    traffic_sides = None
    prof = args.traffic_json or latest_profile()
    if prof and os.path.exists(prof) and args.accum_mode == 0:
        with open(prof) as f:
            pj = json.load(f)
        fresh = {src: pj.get("sources_sha256", {}).get(src) == source_sha256(src)
                 for src in ("als.hip", "tt.hip", "tt_mfma.hip")}
        traffic_src = {"profile": os.path.relpath(prof, ROOT), "kernel_source_matches": fresh["als.hip"]}
        if fresh["als.hip"] and world == 1:
            traffic = pj["als_half_sweep"].get("hbm_bytes_avg_per_launch")
            per = pj["als_half_sweep"].get("hbm_bytes_per_launch_corrected") or []
            if len(per) >= 2:  # launches alternate item, user
                traffic_sides = {"item": sum(per[0::2]) / len(per[0::2]), "user": sum(per[1::2]) / len(per[1::2])}
        if fresh["tt.hip"]:
            tsw = pj.get("tt_adam_sweep", {})
    if tt_iv is not None:
        tiv = pj.get("tt_item_forward_c4", {}) if traffic_src and fresh["tt_mfma.hip"] and world == 1 else {}
        tt_iv["roofline"]["traffic"] = tiv.get("hbm_bytes_avg_per_launch_corrected")
        tt_iv["roofline"]["traffic_note"] = ("HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, "
                                             "scripts/gpu_profile.sh; null when the profile predates csrc/tt_mfma.hip)")
    if tt_train is not None:
        tt_train["roofline"]["traffic"] = tsw.get("hbm_bytes_avg_per_launch_corrected") if tsw else None
        tt_train["roofline"]["traffic_note"] = (
            "HBM bytes per launch of the whole-table Adam sweep (adam_sparse_group4_kernel, rocprofv3 "
            "FETCH_SIZE x2 + WRITE_SIZE, scripts/gpu_profile.sh; null when the profile predates csrc/tt.hip); "
            "achieved above is the whole step's")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(eng, cfg, min(args.cpu_user_rows, n_users), min(args.cpu_item_rows, n_items))

    # BASELINE configs[2] (c3: 10M x 1M, 1 %, rank 64, user-sharded ALS with
    # RCCL all-gathers on 8 GPUs) as a sub-line of every run with >= 8 ranks,
    # after the c2 lines (their buffers freed): the headline stays c2 at every
    # N so the driver's 1/2/4/8 values compare the same workload.
    als_c3 = None
    if world >= CONFIGS["c3"]["min_world"] and args.config != "c3" and args.c3_epochs > 0:
        del eng, csr, csc
        torch.cuda.empty_cache()
        als_c3 = c3_line(world, rank, group, chunks, args.c3_epochs, stream)

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        line = {
            "metric": METRIC,
            "value": args.steps / elapsed,
            "unit": "epochs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (hash-defined interaction matrix generated on device, BASELINE.md §3)",
            "config": {
                "workload": (f"{args.config}: {n_users} users x {n_items} items, density {cfg['density']}, "
                             f"rank {k}, reg 0.1; step = one ALS epoch (item + user half-sweep)"),
                "users": n_users, "items": n_items, "density": cfg["density"], "rank": k,
                "nnz": nnz_user, "nnz_check_csc": nnz_item,
                "shard_nnz_max_over_min": max(per_rank_nnz) / max(1, min(per_rank_nnz)),
                "shard_layout": als["layout"],
                "parallelism": (f"dp{world} (users/items in contiguous parts balanced on nnz + per-row solve cost; "
                                f"user side in {chunks} chunks per rank, each chunk's RCCL all-gather overlapping "
                                f"the next chunk's half-sweep)"
                                if world > 1 else "dp1 (single GPU, no collectives)"),
            },
            "world_size": world,
            "collectives": als["collectives"],
            "roofline": {
                "kernel": "als_half_sweep_f64_kernel (item + user launches)",
                "bound": "mfma",
                "achieved": achieved_tf,
                "peak": F64_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved_tf / F64_MFMA_PEAK_TFLOPS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "traffic_note": ("memory-side bytes per launch from rocprofv3 FETCH_SIZE(x2, gfx950) + WRITE_SIZE, "
                                 "separate PMC passes of this command (scripts/gpu_profile.sh -> profiles/); "
                                 "FETCH_SIZE counts L2 fills from the Infinity Cache as well as HBM: the user "
                                 "side gathers the f64 copy of the item factors (51 MB, Infinity-Cache resident, "
                                 "512 B per rating), so most of its bytes are L3 -> L2 fills, not HBM"),
                "traffic_per_side": traffic_sides,
                "algorithmic_flops_per_launch": flops / 2,
                "avg_launch_ms": (item_ms + user_ms) / 2,
                "kernel_ms_per_epoch": {"item": item_ms, "user": user_ms},
                "gather_view": {"algorithmic_GBps": bytes_ / kern_s / 1e9, "hbm_peak_GBps": HBM_PEAK_GBS,
                                "frac": bytes_ / kern_s / 1e9 / HBM_PEAK_GBS},
            },
            "cpu_baseline": cpu,
            "scoring": scoring,
            "hybrid_top5": hybrid,
            "ingest": ingest,
            "tt_item_vectors_c4": tt_iv,
            "tt_scoring_c4": tt_c4,
            "hybrid_top5_c5": hybrid_c5,
            "tt_train": tt_train,
            "api_hybrid_call": api,
            "als_rank256": als256,
            "als_c3": als_c3,
        }
        attach_counters(line, pj if world == 1 else {}, prof)
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
