set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/c5_prune_diag.py > gpurun_out/r05_c5_diag.txt 2>&1 || { tail -30 gpurun_out/r05_c5_diag.txt; exit 1; }
cat gpurun_out/r05_c5_diag.txt
