#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
HREC_LIB=$PWD/hybrid-als-twotower-recommender_amd/lib/variants/libhrec_hxst.so timeout -k 10 300 python -u scripts/hx_stamps.py > gpurun_out/r05_hx_stamps.log 2>&1 || { tail -30 gpurun_out/r05_hx_stamps.log; exit 1; }
cat gpurun_out/r05_hx_stamps.log
