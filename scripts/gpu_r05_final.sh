# round-5 evidence, part 1: full gpu suite, smoke, the default bench line.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r05_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r05_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r05_gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python -u bench.py > gpurun_out/r05_bench.json 2> gpurun_out/r05_bench.err || { tail -20 gpurun_out/r05_bench.err; exit 1; }
tail -c 300 gpurun_out/r05_bench.json
echo done
