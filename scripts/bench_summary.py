"""Print the headline and every sub-line of a bench JSON line (gpurun_out/bench.json)."""
import json
import sys

d = json.loads(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"], d["roofline"]["kernel_ms_per_epoch"])
for k in ("scoring", "hybrid_top5", "hybrid_top5_c5", "api_hybrid_call", "tt_scoring_c4", "ingest", "tt_train",
          "als_rank256", "tt_item_vectors_c4"):
    v = d.get(k)
    if not v:
        print(k, None)
        continue
    print("==", k, {kk: vv for kk, vv in v.items() if not isinstance(vv, (dict, list)) and kk not in ("note", "steps", "kernel")})
    if "roofline" in v:
        r = v["roofline"]
        print("   roofline", {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in r.items()
                              if kk not in ("stages", "note", "kernel")})
        for s in r.get("stages", []):
            print("     stage", s["kernel"][:70], round(s["avg_launch_ms"], 4), round(s["frac"], 3))
    if "cpu_baseline" in v and v["cpu_baseline"]:
        print("   cpu", v["cpu_baseline"]["value"], v["cpu_baseline"]["unit"])
c4 = d.get("tt_scoring_c4") or {}
for k in ("f32", "bf16", "f32_B1", "bf16_B1", "tower_check"):
    print(k, c4.get(k))
