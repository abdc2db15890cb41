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
