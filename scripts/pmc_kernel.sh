# PMC passes for one kernel of the bench (run via gpurun):
#   bash scripts/pmc_kernel.sh <kernel-substring> [bench args...]
# One rocprofv3 --pmc pass per counter group (no tracing domains).
set -e
K=$1; shift
python -c "import __graft_entry__ as g; g.build()"
mkdir -p gpurun_out/pmck
export TMPDIR=/tmp
A="--no-cpu-baseline --no-ingest --steps 1 --warmup 0 $*"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmck/p$i -o p$i -- python bench.py $A > /dev/null 2> gpurun_out/pmck/p$i.err
done
python - "$K" <<'PY'
import csv, glob, sys, collections
k = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmck/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if k in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for c in sorted(agg):
    v = agg[c]
    print(f"{c:24s} n={len(v):3d} avg={sum(v)/len(v):.4g}")
PY
