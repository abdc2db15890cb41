# Kernel trace of the c5 hybrid line alone (pruned bf16 path): per-kernel
# durations and the gaps between them (eager and HIP-graph replay).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
C5_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o c5 -- python bench.py $C5_ONLY > gpurun_out/prof_c5.json 2> gpurun_out/prof_c5.err
python scripts/trace_gaps.py gpurun_out/prof_c5 > gpurun_out/prof_c5_gaps.txt
tail -60 gpurun_out/prof_c5_gaps.txt
