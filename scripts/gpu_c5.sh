# c5 hybrid: dot/hybrid parity tests, then the c5 + c2-hybrid bench lines only.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dot.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dot_tests.log 2>&1 || { tail -30 gpurun_out/dot_tests.log; exit 1; }
tail -1 gpurun_out/dot_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ingest --c4-items 0 --score-users 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0 > gpurun_out/c5.json 2> gpurun_out/c5.err
python - <<'PY'
import json
d = json.load(open("gpurun_out/c5.json"))
for key in ("hybrid_top5", "hybrid_top5_c5"):
    h = d[key]
    print(key, round(h["ms_per_batch"], 4), "ms", h["launch"])
    for s in h["roofline"]["stages"]:
        print("   ", round(s["avg_launch_ms"] * 1e3, 1), "us", s["kernel"], round(s["frac"], 3))
PY
