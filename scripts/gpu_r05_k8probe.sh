set -e
mkdir -p gpurun_out
timeout -k 10 200 python3 -u scripts/k8_filter_probe.py > gpurun_out/r05_k8probe.txt 2>&1 || { tail -20 gpurun_out/r05_k8probe.txt; exit 1; }
cat gpurun_out/r05_k8probe.txt
