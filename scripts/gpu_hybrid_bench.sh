# GPU: the two hybrid bench lines only (stage breakdown in roofline.stages)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 1 --warmup 0 --score-users 0 --c4-items 0 --tt-steps 0 --no-ingest --api-reps 0 --rank256-epochs 0 --no-cpu-baseline "$@" > gpurun_out/bench_hyb.json 2> gpurun_out/bench_hyb.err || { tail -20 gpurun_out/bench_hyb.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_hyb.json"))
for k in ("hybrid_top5", "hybrid_top5_c5"):
    h = d[k]
    print(k, f"{h['ms_per_batch']*1e3:.1f} us/batch (eager {h['eager_ms_per_batch']*1e3:.1f})", f"{h['pairs_per_s']:.3g} pairs/s")
    for st in h["roofline"]["stages"]:
        print(f"   {st['kernel'][:60]:60s} {st['avg_launch_ms']*1e3:7.1f} us  frac {st['frac']:.3f}")
PY
