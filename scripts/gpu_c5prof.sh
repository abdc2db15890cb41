set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dot.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dot_tests.log 2>&1 || { tail -30 gpurun_out/dot_tests.log; exit 1; }
tail -1 gpurun_out/dot_tests.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof2 -o c5 -- python -u bench.py --no-cpu-baseline --no-ingest --c4-items 0 --score-users 0 --hybrid-users 0 --steps 1 --warmup 0 > gpurun_out/c5prof2.log 2>&1
grep -o '"hybrid_top5_c5.*' gpurun_out/c5prof2.log | head -c 200
