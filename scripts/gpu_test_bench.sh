# GPU: parity tests, then the default bench (one JSON line) -> gpurun_out/
set -e
python -c "import __graft_entry__ as g; g.build()"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 400 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
