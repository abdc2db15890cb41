# Two-stream sparse Adam: all gpu tests, then the tt_train line with the
# phased path on and off.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
TT="--no-cpu-baseline --no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --c5-users 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0"
for r in 1 2; do
  for p in ${MODES:-1 0}; do
    HREC_TT_PHASED=$p timeout -k 10 300 python -u bench.py $TT > gpurun_out/tt_p$p.json 2> gpurun_out/tt_p$p.err
    python -c "import json; d=json.load(open('gpurun_out/tt_p$p.json'))['tt_train']; print('phased=$p', round(d['ms_per_step']*1e3,1), 'us/step', round(d['samples_per_s']))"
  done
done
