# PMC passes for one kernel of an arbitrary command (run via gpurun):
#   bash scripts/pmc_cmd.sh <kernel-substring> <python script> [args...]
# One rocprofv3 --pmc pass per counter group (no tracing domains).
set -e
K=$1; shift
mkdir -p gpurun_out/pmcc
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmcc/p$i -o p$i -- python "$@" > gpurun_out/pmcc/p$i.log 2>&1
done
python - "$K" <<'PY'
import csv, glob, sys, collections
k = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmcc/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if k in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for c in sorted(agg):
    v = agg[c]
    print(f"{c:28s} n={len(v):3d} avg={sum(v)/len(v):.5g}")
PY
