# Hybrid batch cost vs users per batch (c2 exact + c5 bf16 lines only).
set -e
mkdir -p gpurun_out
for u in ${USERS:-64 128 256 512}; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ingest --c4-items 0 --score-users 0 --tt-steps 0 \
    --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0 --c5-users $u --hybrid-users $u > gpurun_out/c5u_$u.json 2> gpurun_out/c5u_$u.err
  python - $u <<'PY'
import json, sys
u = int(sys.argv[1])
d = json.load(open(f"gpurun_out/c5u_{u}.json"))
for k in ("hybrid_top5", "hybrid_top5_c5"):
    h = d[k]
    print(u, k, round(h["ms_per_batch"] * 1e3, 1), "us", round(h["ms_per_batch"] * 1e3 / u, 3), "us/user",
          [round(s["avg_launch_ms"] * 1e3, 1) for s in h["roofline"]["stages"]])
PY
done
