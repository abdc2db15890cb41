# round-3 checks: large-operand + pruned-path tests, then the c5 kernel trace
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dot.py tests/test_gpu_ingest.py -v --timeout 300 --timeout-method thread > gpurun_out/r03_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r03_tests.log | grep -v PASSED | head -20; tail -3 gpurun_out/r03_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash scripts/prof_c5.sh
