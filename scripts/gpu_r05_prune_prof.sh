# kernel trace of the scoring stage (bench with the other lines cut short)
set -e
mkdir -p gpurun_out/prune_prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prune_prof -o run -- python3 bench.py --steps 2 --warmup 1 --c4-items 100000 --c5-users 8 --api-reps 2 --tt-steps 2 --no-ingest --no-cpu-baseline --rank256-epochs 0 --c3-epochs 0 > gpurun_out/prune_prof/bench.json 2> gpurun_out/prune_prof/bench.err || { tail -20 gpurun_out/prune_prof/bench.err; exit 1; }
find gpurun_out/prune_prof -name "*kernel_stats.csv" | head -3
