# Trio ALS variant: half-sweep parity tests on it, then A/B against the base build.
set -e
mkdir -p gpurun_out
HREC_LIB=hybrid-als-twotower-recommender_amd/lib/ab/libhrec_pair8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_core.py -q -x -k "half_sweep or engine" --timeout 120 --timeout-method thread > gpurun_out/trio_tests.log 2>&1 || { tail -30 gpurun_out/trio_tests.log; exit 1; }
tail -3 gpurun_out/trio_tests.log
bash scripts/ab_variants.sh
