# JVM-exact score + top-k: parity tests, timing probe and kernel trace
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_core.py tests/test_gpu_api.py tests/test_gpu_als_wide.py -x -q --timeout 120 --timeout-method thread -k "score or recommend or hybrid or predict" > gpurun_out/score_tests.log 2>&1 || { tail -40 gpurun_out/score_tests.log; exit 1; }
tail -1 gpurun_out/score_tests.log
timeout -k 10 200 python -u scripts/score_quick.py 1024 2>&1 | grep -v amdgpu.ids
bash scripts/prof_score.sh | tail -12
