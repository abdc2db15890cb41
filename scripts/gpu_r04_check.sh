# round-4 check: full gpu suite, the N=1 bench, and the W=2 flow launched by
# bench.py itself (no torchrun; gloo carries the collectives, both ranks on
# device 0), incl. the c3 sub-line's flow at 1/10 scale.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/r04_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err
rc=$?; tail -c 600 gpurun_out/r04_bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r04_bench.err; exit $rc; }
HREC_BENCH_BACKEND=gloo HREC_BENCH_DEVICE=0 HREC_BENCH_C3_REHEARSAL=2:0.1 timeout -k 10 500 python -u bench.py \
  --gpus 2 --steps 3 --warmup 1 --c4-items 2000000 --rank256-epochs 0 > gpurun_out/r04_bench_w2.json 2> gpurun_out/r04_bench_w2.err
rc=$?; tail -c 400 gpurun_out/r04_bench_w2.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/r04_bench_w2.err; exit $rc; }
