# rocprofv3 kernel stats of a short bench run (scoring + ALS), summary to stdout
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pq -o pq -- python bench.py --no-cpu-baseline --steps 1 --warmup 0 "$@" > gpurun_out/pq.json 2> gpurun_out/pq.err
python - <<'PY'
import csv, glob
rows = list(csv.DictReader(open(glob.glob("gpurun_out/pq/**/*kernel_stats.csv", recursive=True)[0])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us x{int(r["Calls"]):3d}  {r["Name"][:110]}')
PY
python -c "import json; d=json.load(open('gpurun_out/pq.json')); print(d['scoring'])"
