set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ingest.py > gpurun_out/ing_tests.log 2>&1 || { tail -30 gpurun_out/ing_tests.log; exit 1; }
tail -1 gpurun_out/ing_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ing -o ing -- python scripts/ingest_probe.py > gpurun_out/ing_probe.log 2>&1
grep -E "ms" gpurun_out/ing_probe.log
python - <<'P'
import csv
for r in csv.DictReader(open('gpurun_out/prof_ing/ing_kernel_stats.csv')):
    if 'sort_down' in r['Name'] or 'sort_up' in r['Name']:
        print("%-70s calls %4s avg %9.1f us" % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))
P
