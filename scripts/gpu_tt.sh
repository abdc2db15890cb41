set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread -k "adam or tt or twotower or dedup" > gpurun_out/tt_tests.log 2>&1 || { tail -40 gpurun_out/tt_tests.log; exit 1; }
tail -1 gpurun_out/tt_tests.log
bash scripts/prof_tt.sh
