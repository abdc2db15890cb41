set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_core.py -m gpu -q -x -k "score_topk" --timeout 240 --timeout-method thread > gpurun_out/r05_prune_tests.log 2>&1 || { tail -40 gpurun_out/r05_prune_tests.log; exit 1; }
tail -2 gpurun_out/r05_prune_tests.log
bash scripts/gpu_r05_scoreq.sh
