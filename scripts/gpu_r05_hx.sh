#!/bin/bash
# Round 5: the exact pruned hybrid (csrc/hybrid_exact.hip) — parity tests,
# the bf16 pruned tests (shared helpers moved to hybrid_common.h), the c2 probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hybrid_exact.py \
  > gpurun_out/r05_hx_tests.log 2>&1 || { tail -40 gpurun_out/r05_hx_tests.log; exit 1; }
tail -3 gpurun_out/r05_hx_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dot.py \
  -k "hybrid_prune or recommender or captured" > gpurun_out/r05_hp_tests.log 2>&1 || { tail -40 gpurun_out/r05_hp_tests.log; exit 1; }
tail -2 gpurun_out/r05_hp_tests.log
timeout -k 10 300 python -u scripts/hx_probe.py > gpurun_out/r05_hx_probe.log 2>&1 || { tail -40 gpurun_out/r05_hx_probe.log; exit 1; }
cat gpurun_out/r05_hx_probe.log
