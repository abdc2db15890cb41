set -e
mkdir -p gpurun_out
HREC_LIB=hybrid-als-twotower-recommender_amd/lib/variants/libhrec_hsstamps.so timeout -k 10 300 python -u scripts/hs_stamps.py > gpurun_out/r05_hs_stamps.txt 2>&1 || { tail -30 gpurun_out/r05_hs_stamps.txt; exit 1; }
cat gpurun_out/r05_hs_stamps.txt
