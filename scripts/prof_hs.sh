# rocprofv3 kernel stats of scripts/hs_quick.py for the ab/ variants given as arguments.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  HREC_LIB=hybrid-als-twotower-recommender_amd/lib/ab/libhrec_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hs_$v -o hs -- python scripts/hs_quick.py 256 > gpurun_out/prof_hs_$v.log 2>&1
  echo "== $v"; tail -1 gpurun_out/prof_hs_$v.log
  python - "$v" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/prof_hs_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"  {float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:80]}")
PY
done
