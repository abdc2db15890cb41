# pruned ALS top-k: parity tests, then the default bench line
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_core.py -m gpu -q -x -k "score_topk" --timeout 240 --timeout-method thread > gpurun_out/r05_prune_tests.log 2>&1 || { tail -40 gpurun_out/r05_prune_tests.log; exit 1; }
tail -2 gpurun_out/r05_prune_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/r05_bench_prune.json 2> gpurun_out/r05_bench_prune.err || { tail -20 gpurun_out/r05_bench_prune.err; exit 1; }
echo done
