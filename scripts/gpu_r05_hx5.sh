#!/bin/bash
# Round 5: exact pruned hybrid + API fast path + sharded ingest — parity, c2 probe, kernel trace, stamps, API parts.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hybrid_exact.py \
  tests/test_gpu_multirank.py::test_als_model_train_two_ranks_matches_one tests/test_gpu_dot.py::test_dot_topk_batch_of_four_vs_five \
  tests/test_gpu_api.py::test_hybrid_device_path_matches_list_path \
  > gpurun_out/r05_hx_tests.log 2>&1 || { tail -40 gpurun_out/r05_hx_tests.log; exit 1; }
tail -2 gpurun_out/r05_hx_tests.log
timeout -k 10 300 python -u scripts/api_parts.py > gpurun_out/r05_api_parts.txt 2>&1 || { tail -20 gpurun_out/r05_api_parts.txt; exit 1; }
cat gpurun_out/r05_api_parts.txt
timeout -k 10 300 python -u scripts/hx_probe.py --reps 10 --analyze > gpurun_out/r05_hx_probe.log 2>&1 || { tail -40 gpurun_out/r05_hx_probe.log; exit 1; }
head -2 gpurun_out/r05_hx_probe.log; grep -A4 stage_ms gpurun_out/r05_hx_probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05_hx_prof -o hx -- python3 scripts/hx_probe.py --reps 10 > gpurun_out/r05_hx_prof.log 2>&1 || { tail -20 gpurun_out/r05_hx_prof.log; exit 1; }
f=$(find gpurun_out/r05_hx_prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f'{r["Name"][:80]:80s} n={r["Calls"]:>5s} avg={float(r["AverageNs"])/1e3:9.1f}us max={float(r["MaxNs"])/1e3:9.1f}us')
PY
HREC_LIB=$PWD/hybrid-als-twotower-recommender_amd/lib/variants/libhrec_hxst.so timeout -k 10 300 python -u scripts/hx_stamps.py > gpurun_out/r05_hx_stamps.log 2>&1 || { tail -30 gpurun_out/r05_hx_stamps.log; exit 1; }
cat gpurun_out/r05_hx_stamps.log
