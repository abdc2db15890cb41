set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dot.py tests/test_gpu_comm.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c5st_tests.log 2>&1 || { tail -40 gpurun_out/c5st_tests.log; exit 1; }
tail -1 gpurun_out/c5st_tests.log
for r in 1 2; do timeout -k 10 200 python -u scripts/c5_probe.py 50 2>&1 | grep -v amdgpu.ids; done
HREC_LIB=hybrid-als-twotower-recommender_amd/lib/variants/libhrec_hsstamps.so timeout -k 10 300 python -u scripts/hs_stamps.py 2>&1 | grep -v amdgpu.ids
