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
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
