# API path check: the api tests, then the default bench line.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/r05_api_tests.log 2>&1 || { tail -30 gpurun_out/r05_api_tests.log; exit 1; }
tail -2 gpurun_out/r05_api_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/r05_bench.json 2> gpurun_out/r05_bench.err || { tail -20 gpurun_out/r05_bench.err; exit 1; }
echo done
