# c5: hybrid tests on the default (stream) kernel, then probe + kernel trace
# for HREC_HS_STREAM=1 and 0
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_dot.py tests/test_gpu_multirank.py -q -x -k "hybrid or prune or recommender" --timeout 150 --timeout-method thread > gpurun_out/c5s_tests.log 2>&1 || { grep -v amdgpu.ids gpurun_out/c5s_tests.log | tail -40; exit 1; }
tail -1 gpurun_out/c5s_tests.log
for st in 1 0; do
  echo "== HREC_HS_STREAM=$st"
  HREC_HS_STREAM=$st timeout -k 10 200 python -u scripts/c5_probe.py 30 2>&1 | grep -v amdgpu.ids
  HREC_HS_STREAM=$st timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5st_$st -o t -- python scripts/c5_probe.py 20 > /dev/null 2>&1
  python scripts/pmc_table.py gpurun_out/c5st_$st --match hp_ | cut -c1-120
  python scripts/pmc_table.py gpurun_out/c5st_$st --match hyb_ | cut -c1-120
done
