#!/bin/bash
# A/B of the K1 partner stagger: c2 epochs through bench.py, two interleaved rounds.
set -o pipefail
mkdir -p gpurun_out/ab
V=hybrid-als-twotower-recommender_amd/lib/variants
for round in 1 2; do
  for n in base stag4 stag8 stag12; do
    HREC_LIB=$V/libhrec_$n.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --c5-users 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0 --steps 3 > gpurun_out/ab/${n}_r${round}.json 2> gpurun_out/ab/${n}_r${round}.err || { tail -5 gpurun_out/ab/${n}_r${round}.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab/${n}_r${round}.json')); print('$n', $round, round(d['value'],3), d['roofline']['kernel_ms_per_epoch'])"
  done
done
