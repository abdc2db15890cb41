set -e
mkdir -p gpurun_out
for t in ${TILINGS:-1}; do
  echo "tiling $t"
  HREC_DOT_TILING=$t timeout -k 10 300 python -u -m pytest tests/test_gpu_dot.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dot_tests.log 2>&1 || { tail -40 gpurun_out/dot_tests.log; exit 1; }
  tail -1 gpurun_out/dot_tests.log
  HREC_DOT_TILING=$t timeout -k 10 300 python -u scripts/dot_quick.py ${DOTARGS:-50000000 1024 128} 2>&1 | grep -v amdgpu.ids
done
