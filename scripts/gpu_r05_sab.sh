# A/B of the pruned ALS top-k's sample size (wave-tile maxima, no score matrix)
set -e
mkdir -p gpurun_out
for v in s8k s16k s32k s8k; do
  HREC_LIB=hybrid-als-twotower-recommender_amd/lib/variants/libhrec_$v.so timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --c4-items 100000 --c5-users 8 --api-reps 2 --tt-steps 2 --no-ingest --no-cpu-baseline --rank256-epochs 0 --c3-epochs 0 --hybrid-users 8 > gpurun_out/r05_sab.json 2> gpurun_out/r05_sab.err || { tail -20 gpurun_out/r05_sab.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r05_sab.json').read().strip().splitlines()[-1]); s=d['scoring']; print(sys.argv[1], round(s['ms_per_batch']*1e3,1), s['pruned_equals_fused'])" $v
done
