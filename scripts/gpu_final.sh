# Round-end evidence: full GPU check (tests, smoke, bench) then the rocprofv3 profile passes.
set -e
bash scripts/gpu_full.sh
bash scripts/gpu_profile.sh > gpurun_out/profile.log 2>&1 || { tail -30 gpurun_out/profile.log; exit 1; }
tail -5 gpurun_out/profile.log
