# SQ/GRBM counter passes for the ALS half-sweep (run via gpurun):
# MFMA busy cycles vs wave cycles vs effective clock. Each pass is its own
# rocprofv3 run (no tracing domains beside --pmc). Stops at the first failure.
set -e
python -c "import __graft_entry__ as g; g.build()"
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
A="--no-cpu-baseline --no-ingest --score-users 0 --hybrid-users 0 --steps 1 --warmup 0 $*"
timeout -k 10 120 rocprofv3 -L > gpurun_out/sq/counters.txt 2>&1 || true
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/sq/p$i -o p$i -- python bench.py $A > gpurun_out/sq/p$i.json 2> gpurun_out/sq/p$i.err
done
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/sq/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "als_half_sweep" in r.get("Kernel_Name", ""):
            agg[(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
by = collections.defaultdict(dict)
for (d, c), v in agg.items():
    by[c][d] = sum(v)
for c in sorted(by):
    print(c, " ".join(f"{by[c][d]:.4g}" for d in sorted(by[c], key=int)))
PY
