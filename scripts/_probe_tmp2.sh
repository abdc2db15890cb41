set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_trained_ranking.py > gpurun_out/trained.log 2>&1 || { tail -40 gpurun_out/trained.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/trained.log | tail -12
bash scripts/_probe_tmp.sh
