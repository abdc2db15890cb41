# c5 pruned hybrid: per-kernel durations (kernel trace) of the probe (an
# optional list of labels runs it once per label)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in ${@:-1}; do
  echo "== run $r"
  timeout -k 10 200 python -u scripts/c5_probe.py 30 2>&1 | grep -v amdgpu.ids
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5tr_$r -o t -- python scripts/c5_probe.py 20 > /dev/null 2>&1
  python scripts/pmc_table.py gpurun_out/c5tr_$r --match hp_ | cut -c1-150
  python scripts/pmc_table.py gpurun_out/c5tr_$r --match hyb_ | cut -c1-150
done
