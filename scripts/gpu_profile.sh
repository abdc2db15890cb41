# rocprofv3 evidence for every bench line (run via gpurun, in two calls):
#   bash scripts/gpu_profile.sh 1   kernel trace of the default bench; ALS / c4 / two-tower passes
#   bash scripts/gpu_profile.sh 2   c5 / c2 exact hybrid / pruned scoring / ingest / rank-256 passes
#   python scripts/summarize_profile.py gpurun_out > profiles/rNN_prof_summary.json
# Per workload group three PMC passes, each its own run (no tracing domains;
# MI355X_MICROARCH.md rocprofv3 PMC slots): FETCH_SIZE, WRITE_SIZE, and
# SQ_VALU_MFMA_BUSY_CYCLES + SQ_BUSY_CYCLES + GRBM_GUI_ACTIVE (MFMA busy).
set -e
python -c "import __graft_entry__ as g; g.build()"
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--no-cpu-baseline --steps 3 --warmup 1"
ONE="--steps 1 --warmup 0 --no-cpu-baseline"
MFMA="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
passes() {  # passes <tag> <args...>: FETCH, WRITE and MFMA passes of one bench subset
  tag=$1; shift
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_$tag -o f$tag -- python bench.py "$@" > /dev/null 2> gpurun_out/prof_fetch_$tag.err
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_$tag -o w$tag -- python bench.py "$@" > /dev/null 2> gpurun_out/prof_write_$tag.err
  timeout -k 10 300 rocprofv3 --pmc $MFMA --output-format csv -d gpurun_out/prof_mfma_$tag -o m$tag -- python bench.py "$@" > /dev/null 2> gpurun_out/prof_mfma_$tag.err
  echo "passes $tag done"
}
NONE="--no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --c5-users 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0"
if [ "$1" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o trace -- python bench.py $A > gpurun_out/prof_bench.json 2> gpurun_out/prof_trace.err
  echo "trace done"
  passes als $A $NONE
  passes c4 $A $NONE --c4-items 50000000
  passes tt $NONE --tt-steps 50 $ONE
fi
if [ "$1" = 2 ]; then
  passes c5 $NONE --c5-users 256 $ONE
  passes hx $NONE --hybrid-users 256 $ONE
  passes score $NONE --score-users 1024 $ONE
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_ing -o fetching -- python scripts/ingest_probe.py > /dev/null 2> gpurun_out/prof_fetch_ing.err
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_ing -o writeing -- python scripts/ingest_probe.py > /dev/null 2> gpurun_out/prof_write_ing.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wide -o wide -- python scripts/wide_quick.py 256 300000 100000 > gpurun_out/prof_wide.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc $MFMA --output-format csv -d gpurun_out/prof_mfma_wide -o mwide -- python scripts/wide_quick.py 256 300000 100000 > /dev/null 2> gpurun_out/prof_mfma_wide.err
  echo "part 2 done"
fi
