# JVM-exact scoring probe + profile + the scoring/top-k GPU tests
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_core.py -k "topk" 2>&1 | tail -3
timeout -k 10 120 python -u scripts/score_quick.py 1024
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sq -o sq -- python scripts/score_quick.py 1024 > gpurun_out/sq.log 2>&1
python - <<'PY'
import csv, glob
rows = list(csv.DictReader(open(glob.glob("gpurun_out/sq/**/*kernel_stats.csv", recursive=True)[0])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'{float(r["AverageNs"])/1e3:10.1f} us x{int(r["Calls"]):3d}  {r["Name"][:100]}')
PY
[ -n "$FULL" ] && timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_core.py tests/test_gpu_dot.py tests/test_gpu_api.py "$@" 2>&1 | tail -3
