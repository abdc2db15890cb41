set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/api_parts.py > gpurun_out/r05_api_parts.txt 2>&1 || { tail -30 gpurun_out/r05_api_parts.txt; exit 1; }
cat gpurun_out/r05_api_parts.txt
