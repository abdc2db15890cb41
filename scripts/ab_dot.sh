set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dot.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dot_tests.log 2>&1 || { tail -40 gpurun_out/dot_tests.log; exit 1; }
tail -1 gpurun_out/dot_tests.log
V=hybrid-als-twotower-recommender_amd/lib/ab
for r in 1 2; do for n in ni2 ni4; do
 echo "== $n"; HREC_LIB=$V/libhrec_$n.so timeout -k 10 200 python -u scripts/dot_quick.py 50000000 1024 128 bf16 2>&1 | grep -v amdgpu.ids
done; done
for n in ni2 ni4; do echo "== $n d256"; HREC_LIB=$V/libhrec_$n.so timeout -k 10 200 python -u scripts/dot_quick.py 100000 256 256 bf16 2>&1 | grep -v amdgpu.ids; done
