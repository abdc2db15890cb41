# ingest at c2 (scripts/ingest_probe.py): kernel trace + SQ counter passes,
# to see where the radix downsweep's cycles go.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ingsq_trace -o t -- python scripts/ingest_probe.py > gpurun_out/ingsq_probe.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/ingsq_sq1 -o sq1 -- python scripts/ingest_probe.py > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/ingsq_sq2 -o sq2 -- python scripts/ingest_probe.py > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/ingsq_fetch -o f -- python scripts/ingest_probe.py > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/ingsq_write -o w -- python scripts/ingest_probe.py > /dev/null 2>&1
grep -v amdgpu.ids gpurun_out/ingsq_probe.log
python scripts/pmc_table.py gpurun_out/ingsq_trace gpurun_out/ingsq_sq1 gpurun_out/ingsq_sq2 gpurun_out/ingsq_fetch gpurun_out/ingsq_write > gpurun_out/ingsq_table.txt
cat gpurun_out/ingsq_table.txt
