# Round 5 ingest: parity tests, the multirank drop-in ingest, the bench ingest line + kernel trace.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_ingest.py tests/test_gpu_multirank.py::test_als_model_train_two_ranks_matches_one tests/test_gpu_core.py > gpurun_out/r05_ingest_tests.log 2>&1 || { tail -30 gpurun_out/r05_ingest_tests.log; exit 1; }
tail -2 gpurun_out/r05_ingest_tests.log
A="--no-cpu-baseline --score-users 0 --hybrid-users 0 --c4-items 0 --c5-users 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0"
timeout -k 10 300 python -u bench.py $A > gpurun_out/r05_ingest_bench.json 2> gpurun_out/r05_ingest_bench.err || { tail -20 gpurun_out/r05_ingest_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r05_ingest_bench.json').read().strip().splitlines()[-1]); i=d['ingest']; print(i['ms'], i['csr_matches_generator'], i['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05_ing_prof -o ing -- python bench.py $A > gpurun_out/r05_ing_prof.log 2>&1
f=$(find gpurun_out/r05_ing_prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:18]:
    print(f'{r["Name"][:80]:80s} n={r["Calls"]:>5s} avg={float(r["AverageNs"])/1e3:9.1f}us')
PY
