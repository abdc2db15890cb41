# A/B of the pruned ALS top-k's sample size (sample users per block 64)
set -e
mkdir -p gpurun_out
for sf in 4096 8192 16384 32768; do
  HREC_PRUNE_SAMPLE=$sf HREC_PRUNE_UB_S=64 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --c4-items 100000 --c5-users 8 --api-reps 2 --tt-steps 2 --no-ingest --no-cpu-baseline --rank256-epochs 0 --c3-epochs 0 --hybrid-users 8 > gpurun_out/r05_ubab.json 2> gpurun_out/r05_ubab.err || { tail -20 gpurun_out/r05_ubab.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r05_ubab.json').read().strip().splitlines()[-1]); s=d['scoring']; print(sys.argv[1], round(s['ms_per_batch']*1e3,1), s['pruned_equals_fused'], s['pairs_per_user'])" $sf
done
