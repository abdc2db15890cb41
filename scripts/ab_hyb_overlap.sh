# A/B of the two-stream score phase of the c2 hybrid top-5 (HREC_HYB_OVERLAP):
# parity tests first, then the bench's hybrid line with the knob off / on (x2).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "hybrid or recommend or captured or sharded" > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
ARGS="--steps 1 --warmup 1 --c4-items 0 --c5-users 0 --no-cpu-baseline --rank256-epochs 0 --api-reps 0 --no-ingest --tt-steps 0"
for v in 0 1 0 1; do
  HREC_HYB_OVERLAP=$v timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1])['hybrid_top5']; print('overlap=$v', d['ms_per_batch'], d.get('eager_ms_per_batch'), d.get('graph_ms_per_batch'))"
done
