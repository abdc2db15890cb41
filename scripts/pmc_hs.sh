# FETCH_SIZE / WRITE_SIZE of hyb_scores_kernel at c5's shape (separate passes).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_hs_$c -o p -- python scripts/hs_quick.py 256 > gpurun_out/pmc_hs_$c.log 2>&1
  python - $c <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/pmc_hs_{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "hyb_scores_kernel" in r["Kernel_Name"]]
print(sys.argv[1], "KiB per launch (avg of", len(v), "):", sum(v) / len(v))
PY
done
