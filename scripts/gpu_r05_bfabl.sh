# bound-filter ablation: trace of the scoring stage per variant
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in abl3 abl4; do
  rm -rf gpurun_out/bfabl_$v
  HREC_LIB=hybrid-als-twotower-recommender_amd/lib/variants/libhrec_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bfabl_$v -o t -- python3 bench.py --steps 1 --warmup 1 --c4-items 100000 --c5-users 8 --api-reps 2 --tt-steps 2 --no-ingest --no-cpu-baseline --rank256-epochs 0 --c3-epochs 0 --hybrid-users 8 > gpurun_out/bfabl_$v.json 2> gpurun_out/bfabl_$v.err || { tail -20 gpurun_out/bfabl_$v.err; exit 1; }
  python3 -c "
import csv,sys
for r in csv.DictReader(open('gpurun_out/bfabl_$v/t_kernel_stats.csv')):
    if 'als_bound_filter' in r['Name']: print('$v', r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
done
python3 -c "import json; d=json.loads(open('gpurun_out/bfabl_abl3.json').read().strip().splitlines()[-1]); print('abl3 equal', d['scoring']['pruned_equals_fused'], d['scoring']['ms_per_batch'])"
