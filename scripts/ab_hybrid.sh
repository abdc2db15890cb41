# A/B the hybrid top-5 path (bench hybrid_top5 only) over the libraries in lib/ab
set -e
mkdir -p gpurun_out/ab
V=hybrid-als-twotower-recommender_amd/lib/ab
A="--steps 1 --warmup 0 --no-cpu-baseline --no-ingest --score-users 0 --c4-items 0 --c5-users 0 --tt-steps 0"
timeout -k 10 300 python -u -m pytest tests/test_gpu_core.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread -k "hybrid or fusion" > gpurun_out/hy_tests.log 2>&1 || { tail -30 gpurun_out/hy_tests.log; exit 1; }
tail -1 gpurun_out/hy_tests.log
for round in 1 2; do
  for lib in $V/*.so; do
    n=$(basename $lib .so)
    HREC_LIB=$lib timeout -k 10 200 python bench.py $A > gpurun_out/ab/${n}_h${round}.json
    python -c "import json; d=json.load(open('gpurun_out/ab/${n}_h${round}.json'))['hybrid_top5']; print('$n', $round, round(d['ms_per_batch'],4))"
  done
done
