# A/B the ab/ variants on the tt_train line (two-stream mode 1; mode 0 = one stream).
set -e
mkdir -p gpurun_out/ab
TT="--no-cpu-baseline --no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --c5-users 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0"
for r in 1 2; do
  for lib in hybrid-als-twotower-recommender_amd/lib/ab/*.so; do
    n=$(basename $lib .so)
    for p in ${MODES:-1}; do
      HREC_LIB=$lib HREC_TT_PHASED=$p timeout -k 10 300 python -u bench.py $TT > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err
      python -c "import json; d=json.load(open('gpurun_out/ab/$n.json'))['tt_train']; print('$n mode=$p', round(d['ms_per_step']*1e3,1), 'us/step')"
    done
  done
done
