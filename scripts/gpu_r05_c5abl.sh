# c5 phase-1 ablations (timing-only builds): hyb_scores_kernel<256, 4, 1> with no min/max (abl2), staging only (abl3), head.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/hybrid-als-twotower-recommender_amd/lib/variants
for n in head abl2 abl3; do
  if [ $n = head ]; then unset HREC_LIB; else export HREC_LIB=$V/libhrec_$n.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5abl_$n -o k -- python scripts/c5_probe.py 20 > gpurun_out/c5abl_$n.log 2>&1 || true
  f=$(find gpurun_out/c5abl_$n -name '*kernel_stats.csv' | head -1)
  python3 - "$n" "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[2])):
    if "hyb_scores" in r["Name"] or "hp_" in r["Name"] or "dot_res" in r["Name"]:
        print(sys.argv[1], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
done
