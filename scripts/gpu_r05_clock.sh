#!/bin/bash
# the clock the bf16 c4 dot_res_kernel<true, 128, ...> holds at B = 1024
# (GRBM_GUI_ACTIVE / 8 XCDs / kernel time; MI355X_MICROARCH.md "DVFS give-back").
set -o pipefail
mkdir -p gpurun_out/clk
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/clk/trace -o t -- python scripts/dot_quick.py 50000000 1024 128 bf16 > gpurun_out/clk/trace.log 2>&1 || { tail -5 gpurun_out/clk/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/clk/pmc -o p -- python scripts/dot_quick.py 50000000 1024 128 bf16 > gpurun_out/clk/pmc.log 2>&1 || { tail -5 gpurun_out/clk/pmc.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, json
k = "dot_res_kernel<true, 128"
dur = []
for f in glob.glob("gpurun_out/clk/trace/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if k in r["Kernel_Name"]:
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/clk/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if k in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
t = sum(dur) / len(dur)
out = {"kernel": k, "launches": len(dur), "avg_s": t}
for c, v in agg.items():
    out[c + "_avg"] = sum(v) / len(v)
if "GRBM_GUI_ACTIVE_avg" in out:
    out["clock_GHz_grbm"] = out["GRBM_GUI_ACTIVE_avg"] / 8 / t / 1e9
print(json.dumps(out, indent=1))
PY
