# c5 pruned hybrid: parity tests, then the batch time with the HS_FILTER
# filter (default) and the round-3 K8 filter (HREC_HP_FILTER=0), twice each.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dot.py tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c5ab_tests.log 2>&1 || { tail -40 gpurun_out/c5ab_tests.log; exit 1; }
tail -1 gpurun_out/c5ab_tests.log
for r in 1 2; do
  for f in 1 0; do echo "HREC_HP_FILTER=$f"; HREC_HP_FILTER=$f timeout -k 10 200 python -u scripts/c5_probe.py 50 2>&1 | grep -v amdgpu.ids; done
done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5ab_trace -o t -- python scripts/c5_probe.py 20 > /dev/null 2>&1
python scripts/pmc_table.py gpurun_out/c5ab_trace --match hrec
