# ALS half-sweep parity tests on the default library, then the A/B variants.
set -e
python -c "import __graft_entry__ as g; g.build()"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_core.py -q -x -k "half_sweep or engine" > gpurun_out/als_tests.log 2>&1 || { tail -30 gpurun_out/als_tests.log; exit 1; }
tail -3 gpurun_out/als_tests.log
bash scripts/ab_variants.sh
