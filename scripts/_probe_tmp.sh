set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dot.py tests/test_gpu_multirank.py tests/test_gpu_api.py > gpurun_out/dot_tests.log 2>&1 || { tail -30 gpurun_out/dot_tests.log; exit 1; }
tail -1 gpurun_out/dot_tests.log
C5_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0 --no-cpu-baseline"
for i in 1 2; do
timeout -k 10 300 python bench.py $C5_ONLY > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err
python scripts/bench_summary.py gpurun_out/c5_bench.json > gpurun_out/c5_sum.txt 2>&1 || true
grep -A3 "hybrid_top5_c5" gpurun_out/c5_sum.txt | cut -c1-250
done
