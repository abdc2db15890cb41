# Kernel trace of the two-tower train step only (bench tt_train line)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tt -o tt -- python bench.py --steps 1 --warmup 0 --score-users 0 --hybrid-users 0 --c5-users 0 --c4-items 0 --no-ingest --api-reps 0 --rank256-epochs 0 --no-cpu-baseline --tt-steps 200 > gpurun_out/prof_tt.json 2> gpurun_out/prof_tt.err
python - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof_tt/**/*kernel_stats.csv", recursive=True):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:16]:
        print(f'{r["Name"][:70]:70s} calls={r["Calls"]:>6s} avg_us={float(r["AverageNs"])/1e3:8.2f} pct={float(r["Percentage"]):6.2f}')
PY
# one step's timeline (the last untouched-rows sweep and its neighbours)
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_tt/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
sw = [r for r in rows if "adam_sparse_group4_kernel<true>" in r["Kernel_Name"]]
if sw:
    s0, s1 = int(sw[-2]["Start_Timestamp"]), int(sw[-1]["Start_Timestamp"])
    for r in rows:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s0 - 20000 <= a <= s1:
            print(f'{(a - s0) / 1e3:8.1f} {(b - s0) / 1e3:8.1f} {(b - a) / 1e3:7.1f} q{r.get("Queue_Id", "?")} {r["Kernel_Name"][:60]}')
PY
