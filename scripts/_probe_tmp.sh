set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dot.py tests/test_gpu_multirank.py > gpurun_out/dot_tests.log 2>&1 || { tail -30 gpurun_out/dot_tests.log; exit 1; }
tail -1 gpurun_out/dot_tests.log
C45="--no-ingest --score-users 0 --hybrid-users 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 500 python bench.py $C45 > gpurun_out/c45_bench.json 2> gpurun_out/c45_bench.err
python scripts/bench_summary.py gpurun_out/c45_bench.json > gpurun_out/c45_sum.txt 2>&1 || true
grep -E "hybrid_top5_c5|^f32|^bf16" gpurun_out/c45_sum.txt | cut -c1-400
