set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dotprof -o dot -- python -u scripts/dot_quick.py 50000000 1024 128 bf16 > gpurun_out/dotprof.log 2>&1
cat gpurun_out/dotprof.log | grep -v amdgpu.ids
f=$(find gpurun_out/dotprof -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -20
