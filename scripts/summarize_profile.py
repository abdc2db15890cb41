"""Summarise rocprofv3 CSVs (kernel stats + FETCH_SIZE/WRITE_SIZE passes) for
the dominant kernel. FETCH_SIZE / WRITE_SIZE are KiB per dispatch; on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) streaming reads, so it
is doubled (MI355X_MICROARCH.md §HBM). The half-sweep's gathers are 16-B
loads per lane; its CSR streams are 4-B loads (uncalibrated: reported raw
and doubled)."""
import csv
import glob
import json
import os
import sys

KERNEL = "als_half_sweep_f64_kernel"


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def source_hashes():
    """sha256 of every kernel source at profile time: bench.py compares the
    entry of the kernel it reports against the tree it runs from, so a
    roofline.traffic read from a stale profile is flagged, not silently used."""
    import hashlib

    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hybrid-als-twotower-recommender_amd",
                        "csrc")
    out = {}
    for f in sorted(os.listdir(root)):
        if f.endswith((".hip", ".h")):
            with open(os.path.join(root, f), "rb") as fh:
                out[f] = hashlib.sha256(fh.read()).hexdigest()
    return out


def main(base):
    stats = rows(os.path.join(base, "prof_trace", "**", "*kernel_stats.csv"))
    top = sorted(stats, key=lambda r: -float(r["TotalDurationNs"]))[:8]
    res = {"kernel_stats_top": [{"name": r["Name"][:120], "calls": int(r["Calls"]),
                                 "avg_ms": float(r["AverageNs"]) / 1e6, "pct": float(r["Percentage"])}
                                for r in top]}
    trace = rows(os.path.join(base, "prof_trace", "**", "*kernel_trace.csv"))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace if KERNEL in r["Kernel_Name"]]
    res["als_half_sweep"] = {"launches": len(durs), "avg_ms": sum(durs) / max(len(durs), 1),
                             "durations_ms": durs}
    for name, sub in (("FETCH_SIZE", "prof_fetch"), ("WRITE_SIZE", "prof_write")):
        pmc = rows(os.path.join(base, sub, "**", "*counter_collection.csv"))
        vals = [float(r["Counter_Value"]) for r in pmc
                if KERNEL in r.get("Kernel_Name", "") and r.get("Counter_Name") == name]
        res["als_half_sweep"][name + "_KiB_per_launch"] = vals
    f = res["als_half_sweep"]["FETCH_SIZE_KiB_per_launch"]
    w = res["als_half_sweep"]["WRITE_SIZE_KiB_per_launch"]
    if f and w:
        n = min(len(f), len(w))
        per = [(2 * f[i] + w[i]) * 1024 for i in range(n)]
        res["als_half_sweep"]["hbm_bytes_per_launch_corrected"] = per
        res["als_half_sweep"]["hbm_bytes_avg_per_launch"] = sum(per) / n
    # c4 two-tower scoring: the fused dot + filter launches (FILTER = true) of
    # the f32 and bf16 passes, HIP-trace durations and FETCH_SIZE (x2: 16-B
    # lane loads) per launch
    import re

    def is_filter(name):
        m = re.search(r"dot_(res|tile)_kernel<(\w+), (\d+), (\w+)", name)
        return m and m.group(4) == "true"

    dot = {}
    for r in trace:
        if is_filter(r["Kernel_Name"]):
            dt = "bf16" if "dot_res_kernel<true" in r["Kernel_Name"] or "dot_tile_kernel<true" in r["Kernel_Name"] \
                else "f32"
            dot.setdefault(dt, {"durations_ms": []})["durations_ms"].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for dt, v in dot.items():
        v["avg_ms"] = sum(v["durations_ms"]) / len(v["durations_ms"])
    for r in rows(os.path.join(base, "prof_fetch_c4", "**", "*counter_collection.csv")):
        if is_filter(r.get("Kernel_Name", "")) and r.get("Counter_Name") == "FETCH_SIZE":
            dt = "bf16" if "kernel<true" in r["Kernel_Name"] else "f32"
            dot.setdefault(dt, {}).setdefault("FETCH_SIZE_KiB_per_launch", []).append(float(r["Counter_Value"]))
    for dt, v in dot.items():
        f = v.get("FETCH_SIZE_KiB_per_launch")
        if f:
            v["hbm_read_bytes_avg_per_launch_corrected"] = 2 * 1024 * sum(f) / len(f)
    res["dot_topk_c4_filter"] = dot
    # two-tower train step: grouped whole-table Adam sweep (all 4 tables per
    # launch; 1.69 GB algorithmic per launch at c2's tables, d = 64)
    tk = "adam_sparse_group4_kernel"
    td = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace if tk in r["Kernel_Name"]]
    tt = {"launches": len(td), "avg_ms": sum(td) / max(len(td), 1)}
    for name, sub in (("FETCH_SIZE", "prof_fetch_tt"), ("WRITE_SIZE", "prof_write_tt")):
        vals = [float(r["Counter_Value"]) for r in rows(os.path.join(base, sub, "**", "*counter_collection.csv"))
                if tk in r.get("Kernel_Name", "") and r.get("Counter_Name") == name]
        if vals:
            tt[name + "_KiB_avg_per_launch"] = sum(vals) / len(vals)
    if "FETCH_SIZE_KiB_avg_per_launch" in tt and "WRITE_SIZE_KiB_avg_per_launch" in tt:
        tt["hbm_bytes_avg_per_launch_corrected"] = 1024 * (2 * tt["FETCH_SIZE_KiB_avg_per_launch"] +
                                                           tt["WRITE_SIZE_KiB_avg_per_launch"])
    res["tt_adam_sweep"] = tt
    # JVM-exact ALS score + filter (the scoring half of the metric)
    sd = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace
          if "als_score_fast_kernel<16, true>" in r["Kernel_Name"]]
    if sd:
        res["als_score_filter"] = {"launches": len(sd), "avg_ms": sum(sd) / len(sd)}
    # the pruned ALS top-k (K2p, the bench's scoring line): trace averages per kernel
    pk = {}
    for key in ("als_prune_user_kernel", "als_bound_filter_kernel<64, true>", "sample_threshold_kernel",
                "als_prune_thr_kernel", "als_bound_filter_kernel<64, false>", "als_rescore_topk_kernel<8>"):
        dd = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace if key in r["Kernel_Name"]]
        if dd:
            pk[key] = {"launches": len(dd), "avg_ms": sum(dd) / len(dd)}
    if pk:
        res["als_score_pruned"] = pk
    wide = rows(os.path.join(base, "prof_wide", "**", "*kernel_trace.csv"))
    wd = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in wide
          if "als_half_sweep_wide_kernel" in r["Kernel_Name"]]
    if wd:
        res["als_half_sweep_wide_rank256"] = {"launches": len(wd), "durations_ms": wd,
                                              "workload": "scripts/wide_quick.py 256 300000 100000 (item, user)"}
    # c4 item-vector precompute (K4m, tt_item_forward_mfma_kernel at d = 128
    # over 50M items): trace durations + FETCH/WRITE passes (x2 on FETCH:
    # 16-B lane loads)
    kf = "tt_item_forward_mfma_kernel<8, 8, true, false, 16, true>"
    fd = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace if kf in r["Kernel_Name"]]
    tf = {"launches": len(fd), "avg_ms": sum(fd) / max(len(fd), 1)}
    for name, sub in (("FETCH_SIZE", "prof_fetch_c4"), ("WRITE_SIZE", "prof_write_c4")):
        vals = [float(r["Counter_Value"]) for r in rows(os.path.join(base, sub, "**", "*counter_collection.csv"))
                if kf in r.get("Kernel_Name", "") and r.get("Counter_Name") == name]
        if vals:
            tf[name + "_KiB_avg_per_launch"] = sum(vals) / len(vals)
    if "FETCH_SIZE_KiB_avg_per_launch" in tf and "WRITE_SIZE_KiB_avg_per_launch" in tf:
        tf["hbm_bytes_avg_per_launch_corrected"] = 1024 * (2 * tf["FETCH_SIZE_KiB_avg_per_launch"] +
                                                           tf["WRITE_SIZE_KiB_avg_per_launch"])
    res["tt_item_forward_c4"] = tf

    # c5 pruned hybrid and ingest: per kernel, trace average + PMC bytes per
    # launch (FETCH x 2: 16-B lane loads)
    def per_kernel(keys, fetch_sub, write_sub):
        out = {}
        for k in keys:
            d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace if k in r["Kernel_Name"]]
            e = {"launches": len(d), "avg_ms": sum(d) / max(len(d), 1)}
            for name, sub in (("FETCH_SIZE", fetch_sub), ("WRITE_SIZE", write_sub)):
                vals = [float(r["Counter_Value"]) for r in rows(os.path.join(base, sub, "**", "*counter_collection.csv"))
                        if k in r.get("Kernel_Name", "") and r.get("Counter_Name") == name]
                if vals:
                    e[name + "_KiB_avg_per_launch"] = sum(vals) / len(vals)
            if "FETCH_SIZE_KiB_avg_per_launch" in e and "WRITE_SIZE_KiB_avg_per_launch" in e:
                e["hbm_bytes_avg_per_launch_corrected"] = 1024 * (2 * e["FETCH_SIZE_KiB_avg_per_launch"] +
                                                                  e["WRITE_SIZE_KiB_avg_per_launch"])
            out[k] = e
        return out

    # every instantiation of the batch's kernels (matched by base name: the
    # r04 keys named one template each and missed hyb_scores_kernel<256, 4, 2>
    # and hp_bound_kernel<256, true>); batch bytes = sum over kernels of the
    # average bytes per launch x launches per batch (hp_user_ops_kernel runs
    # once per batch)
    bases = ["hp_user_ops_kernel", "hyb_scores_kernel<", "hyb_mm_reduce_kernel", "hp_bound_kernel<",
             "dot_res_kernel<true, 256", "hp_cand_topk_kernel<"]
    names = sorted({r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hrec::", "") for r in trace
                    if any(b in r["Kernel_Name"] for b in bases)})
    c5 = per_kernel(names, "prof_fetch_c5", "prof_write_c5")
    n_batches = max(next((e["launches"] for k, e in c5.items() if k.startswith("hp_user_ops_kernel")), 1), 1)
    tot = sum(e.get("hbm_bytes_avg_per_launch_corrected", 0.0) * e["launches"] for e in c5.values()) / n_batches
    c5["batches_in_profile"] = n_batches
    c5["batch_hbm_bytes_corrected"] = tot
    c5["no_store_bytes"] = 102.4e6
    c5["traffic_over_no_store"] = tot / 102.4e6
    res["c5_pruned_hybrid"] = c5
    # c2 exact pruned hybrid (csrc/hybrid_exact.hip): every hx_ kernel
    hx_names = sorted({r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hrec::", "") for r in trace
                       if "hx_" in r["Kernel_Name"]})
    res["c2_exact_hybrid"] = per_kernel(hx_names, "prof_fetch_hx", "prof_write_hx")
    res["ingest"] = per_kernel(["mark_present_kernel", "codes_from_rank_kernel", "mark_bits_kernel",
                                "codes_bits_kernel", "descent_kernel", "copy_entries_kernel",
                                "indptr_from_sorted_kernel", "sort_upsweep_kernel",
                                "sort_downsweep_kernel<true, false>", "sort_downsweep_kernel<false, true>"],
                               "prof_fetch_ing", "prof_write_ing")
    res["kernels"] = per_kernel_counters(base, trace, wide)
    res["sources_sha256"] = source_hashes()
    print(json.dumps(res, indent=1))


def kname(name):
    return name.split("(")[0].replace("void ", "").replace("hrec::", "").strip()


N_SIMD = 1024  # 256 CUs x 4 SIMDs


def per_kernel_counters(base, trace, wide):
    """Every kernel of every pass, by template instantiation: trace average
    duration, HBM bytes per dispatch (FETCH_SIZE x2 + WRITE_SIZE, KiB units,
    gfx950 16-B-load correction) and the MFMA-busy fraction per dispatch:
    SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) (GRBM counts
    every XCD's cycles; the MFMA counter every SIMD's busy cycles; reads low on
    dispatches shorter than ~0.3 ms, MI355X_MICROARCH.md DVFS note), with the
    effective clock GRBM_GUI_ACTIVE / 8 / trace duration."""
    import collections

    out = collections.defaultdict(dict)
    dur = collections.defaultdict(list)
    for r in trace + wide:
        dur[kname(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for k, v in dur.items():
        out[k]["launches_in_trace"] = len(v)
        out[k]["avg_ms"] = sum(v) / len(v)
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    grids = collections.defaultdict(dict)  # kernel -> (pass, dispatch) -> grid size
    for sub in glob.glob(os.path.join(base, "prof_*")):
        if os.path.basename(sub).startswith(("prof_fetch", "prof_write", "prof_mfma")) and os.path.isdir(sub):
            for r in rows(os.path.join(sub, "**", "*counter_collection.csv")):
                kn = kname(r.get("Kernel_Name", ""))
                vals[kn][r.get("Counter_Name")].append(((sub, r.get("Dispatch_Id")), float(r["Counter_Value"])))
                grids[kn][(sub, r.get("Dispatch_Id"))] = int(r.get("Grid_Size") or 0)
    for k, cs in vals.items():
        e = out[k]
        f = [v for _, v in cs.get("FETCH_SIZE", [])]
        w = [v for _, v in cs.get("WRITE_SIZE", [])]
        if f:
            e["FETCH_SIZE_KiB_avg"] = sum(f) / len(f)
        if w:
            e["WRITE_SIZE_KiB_avg"] = sum(w) / len(w)
        if f and w:
            e["hbm_bytes_per_dispatch_corrected"] = 1024 * (2 * e["FETCH_SIZE_KiB_avg"] + e["WRITE_SIZE_KiB_avg"])
        mb = dict(cs.get("SQ_VALU_MFMA_BUSY_CYCLES", []))
        gr = dict(cs.get("GRBM_GUI_ACTIVE", []))
        ds = [d for d in mb if d in gr and gr[d] > 0]
        if ds:
            # time-weighted (sum of busy cycles over sum of SIMD cycles): the
            # long dispatches dominate; per launch shape (grid size) as well,
            # since one kernel serves batches of 1 and of 1024 users
            e["mfma_busy_frac"] = sum(mb[d] for d in ds) / sum(gr[d] / 8 * N_SIMD for d in ds)
            e["mfma_busy_dispatches"] = len(ds)
            by = collections.defaultdict(list)
            for d in ds:
                by[grids[k].get(d, 0)].append(d)
            if len(by) > 1:
                e["mfma_busy_by_grid"] = {
                    str(gsz): {"dispatches": len(dd), "mfma_busy_frac":
                               sum(mb[d] for d in dd) / sum(gr[d] / 8 * N_SIMD for d in dd),
                               "grbm_cycles_per_xcd_avg": sum(gr[d] for d in dd) / len(dd) / 8}
                    for gsz, dd in sorted(by.items())}
            if e.get("avg_ms"):
                e["eff_clock_GHz"] = sum(gr[d] for d in ds) / len(ds) / 8 / (e["avg_ms"] * 1e6)
    return dict(out)


if __name__ == "__main__":
    main(sys.argv[1])
