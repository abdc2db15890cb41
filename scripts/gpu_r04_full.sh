# round-4 check at HEAD: full gpu suite, smoke, the N=1 bench (driver args),
# then the c5 stamps diagnostic build.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/r04_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err
rc=$?; tail -c 300 gpurun_out/r04_bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r04_bench.err; exit $rc; }
HREC_LIB=hybrid-als-twotower-recommender_amd/lib/variants/libhrec_hsstamps.so timeout -k 10 300 python -u scripts/hs_stamps.py 2>&1 | grep -v amdgpu.ids
