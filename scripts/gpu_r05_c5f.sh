# c5 filter with live-user compaction: parity tests, diag timing, bench
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dot.py tests/test_gpu_multirank.py -m gpu -q -x -k "prune or bf16 or recommender or hybrid" --timeout 240 --timeout-method thread > gpurun_out/r05_c5f_tests.log 2>&1 || { tail -30 gpurun_out/r05_c5f_tests.log; exit 1; }
tail -2 gpurun_out/r05_c5f_tests.log
timeout -k 10 300 python -u scripts/c5_prune_diag.py > gpurun_out/r05_c5_diag.txt 2>&1 || { tail -30 gpurun_out/r05_c5_diag.txt; exit 1; }
tail -3 gpurun_out/r05_c5_diag.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r05_bench_c5f.json 2> gpurun_out/r05_bench_c5f.err || { tail -20 gpurun_out/r05_bench_c5f.err; exit 1; }
echo done
