# quick scoring-line check (other bench lines cut short)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --c4-items 100000 --c5-users 8 --api-reps 2 --tt-steps 2 --no-ingest --no-cpu-baseline --rank256-epochs 0 --c3-epochs 0 > gpurun_out/r05_scoreq.json 2> gpurun_out/r05_scoreq.err || { tail -20 gpurun_out/r05_scoreq.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r05_scoreq.json').read().strip().splitlines()[-1]); s=d['scoring']; print({k: s[k] for k in ('ms_per_batch','fused_ms_per_batch','pruned_equals_fused','pairs_per_user')})"
