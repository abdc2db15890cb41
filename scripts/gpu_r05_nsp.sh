# A/B: seed pairs scanned beside the extremes (HREC_HX_NSP cap), c2 hybrid probe.
set -e
mkdir -p gpurun_out
V=hybrid-als-twotower-recommender_amd/lib/variants
for r in 1 2; do
  for n in nsp1 nsp2 nsp4 head; do
    if [ $n = head ]; then L=""; else L="HREC_LIB=$PWD/$V/libhrec_$n.so"; fi
    env $L timeout -k 10 200 python -u scripts/hx_probe.py --reps 20 > gpurun_out/nsp_$n.log 2>&1 || { tail -20 gpurun_out/nsp_$n.log; exit 1; }
    python3 - "$n" gpurun_out/nsp_$n.log <<'PY'
import json, sys
L = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{\"")]
for d in L:
    for k, v in d.items():
        print(sys.argv[1], k, v["bit_identical"], round(v["pruned_eager_ms"], 4), round(v["pruned_graph_ms"], 4), v["groups_topk"])
PY
  done
done
