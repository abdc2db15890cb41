# round-4 evidence, part 1: full gpu suite, smoke, the default bench line,
# and the kernel trace of the bench (+ the rank-256 probe).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r04_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r04_gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python -u bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err || { tail -20 gpurun_out/r04_bench.err; exit 1; }
tail -c 200 gpurun_out/r04_bench.json
A="--no-cpu-baseline --steps 3 --warmup 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o trace -- python bench.py $A > gpurun_out/prof_bench.json 2> gpurun_out/prof_trace.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wide -o wide -- python scripts/wide_quick.py 256 300000 100000 > gpurun_out/prof_wide.log 2>&1
echo done
