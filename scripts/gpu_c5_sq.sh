# c5 pruned hybrid: kernel trace + SQ / memory counter passes of the probe.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/c5_probe.py 50 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5sq_trace -o t -- python scripts/c5_probe.py 20 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --output-format csv -d gpurun_out/c5sq_sq -o sq -- python scripts/c5_probe.py 5 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c5sq_fetch -o f -- python scripts/c5_probe.py 5 > /dev/null 2>&1
python scripts/pmc_table.py gpurun_out/c5sq_trace gpurun_out/c5sq_sq gpurun_out/c5sq_fetch > gpurun_out/c5sq_table.txt
cat gpurun_out/c5sq_table.txt
# c4 one-user GEMV (csrc/dot_gemv.hip): kernel trace + FETCH_SIZE pass
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gemv_trace -o t -- python scripts/gemv_probe.py > gpurun_out/gemv_probe.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/gemv_fetch -o f -- python scripts/gemv_probe.py > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/gemv_write -o w -- python scripts/gemv_probe.py > /dev/null 2>&1
grep -v amdgpu.ids gpurun_out/gemv_probe.log
python scripts/pmc_table.py gpurun_out/gemv_trace gpurun_out/gemv_fetch gpurun_out/gemv_write --match dot_ > gpurun_out/gemv_table.txt
cat gpurun_out/gemv_table.txt
