# W > 1 bench flow rehearsed on ONE GPU: gloo carries the collectives, every
# rank on device 0 (RCCL refuses two ranks per device). Checks that the
# driver's multi-GPU bench (RCCL, one GPU per rank) has no host-side fault.
set -e
mkdir -p gpurun_out
export HREC_BENCH_BACKEND=gloo HREC_BENCH_DEVICE=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${W:-2} --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus ${W:-2} --steps 3 --warmup 1 ${BENCH_ARGS:-} \
  > gpurun_out/bench_w${W:-2}.json 2> gpurun_out/bench_w${W:-2}.err
cat gpurun_out/bench_w${W:-2}.json
