# PMC passes for the dot_tile_kernel FILTER launches (run via gpurun).
set -e
mkdir -p gpurun_out/dotpmc
export TMPDIR=/tmp
i=0
export HREC_DOT_TILING=${HREC_DOT_TILING:-2}
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/dotpmc/p$i -o p$i -- python scripts/dot_quick.py ${DOTARGS:-10000000 1024 128 bf16} > gpurun_out/dotpmc/p$i.log 2>&1
done
python - <<'PY'
import csv, glob, collections, re
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/dotpmc/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"dot_(res|tile)_kernel<(\w+), (\d+), (\w+)", r.get("Kernel_Name", ""))
        if m and m.group(4) == "true":
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for c in sorted(agg):
    v = agg[c]
    print(f"{c:32s} n={len(v):3d} avg={sum(v)/len(v):.5g}")
PY
