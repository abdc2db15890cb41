set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ingest.py tests/test_gpu_dot.py -k "ingest or coo or csr or encode or prune or hybrid or recommender or filter" > gpurun_out/r_tests.log 2>&1 || { tail -30 gpurun_out/r_tests.log; exit 1; }
tail -1 gpurun_out/r_tests.log
C5_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 python bench.py $C5_ONLY > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err
python scripts/bench_summary.py gpurun_out/c5_bench.json > gpurun_out/c5_sum.txt 2>&1; grep -A3 "hybrid_top5_c5" gpurun_out/c5_sum.txt || true
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ing -o ing -- python scripts/ingest_probe.py > gpurun_out/ing_probe.log 2>&1
grep -E "ms" gpurun_out/ing_probe.log
python - <<'P'
import csv
for r in csv.DictReader(open('gpurun_out/prof_ing/ing_kernel_stats.csv')):
    if 'sort_' in r['Name'] or 'mark' in r['Name'] or 'codes_' in r['Name'] or 'indptr' in r['Name'] or 'copy_entries' in r['Name'] or 'descent' in r['Name']:
        print("%-70s calls %4s avg %9.1f us" % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))
P
