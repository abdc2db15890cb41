set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_als_wide.py -x -v --timeout 120 --timeout-method thread > gpurun_out/wide_tests.log 2>&1 || { tail -60 gpurun_out/wide_tests.log; exit 1; }
tail -15 gpurun_out/wide_tests.log
