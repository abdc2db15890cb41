# A/B the ALS half-sweep variants on one GPU (two interleaved rounds).
set -e
mkdir -p gpurun_out/ab
V=hybrid-als-twotower-recommender_amd/lib/ab
for round in 1 2; do
  for lib in $V/*.so; do
    n=$(basename $lib .so)
    HREC_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --c5-users 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0 --steps 3 --accum-mode ${MODE:-0} > gpurun_out/ab/${n}_r${round}.json
    python -c "import json,sys; d=json.load(open('gpurun_out/ab/${n}_r${round}.json')); print('$n', $round, round(d['value'],3), d['roofline']['kernel_ms_per_epoch'])"
  done
done
