# Kernel trace of the hybrid bench lines only
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hyb -o hyb -- python bench.py --steps 1 --warmup 0 --score-users 0 --c4-items 0 --tt-steps 0 --no-ingest --api-reps 0 --rank256-epochs 0 --no-cpu-baseline "$@" > gpurun_out/prof_hyb.json 2> gpurun_out/prof_hyb.err
python - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof_hyb/**/*kernel_stats.csv", recursive=True):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:22]:
        print(f'{r["Name"][:90]:90s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.2f}')
PY
