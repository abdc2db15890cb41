# two-tower training step: bench line (tt_train only) + rocprofv3 kernel stats
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
A="--steps 1 --warmup 0 --no-cpu-baseline --no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --c5-users 0"
timeout -k 10 300 python bench.py $A > gpurun_out/tt.json
python -c "import json; print(json.load(open('gpurun_out/tt.json'))['tt_train'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ptt -o ptt -- python bench.py $A > /dev/null 2> gpurun_out/ptt.err
python - <<'PY'
import csv, glob
rows = list(csv.DictReader(open(glob.glob("gpurun_out/ptt/**/*kernel_stats.csv", recursive=True)[0])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us x{int(r["Calls"]):4d}  {r["Name"][:100]}')
PY
