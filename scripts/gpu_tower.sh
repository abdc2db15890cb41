# GPU: two-tower tests (item tower on MFMA) + the c4 item-vector / scoring lines only
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py -x -q -k "tt_ or twotower" --timeout 300 --timeout-method thread > gpurun_out/tower_tests.log 2>&1 || { tail -40 gpurun_out/tower_tests.log; exit 1; }
tail -2 gpurun_out/tower_tests.log
timeout -k 10 400 python bench.py --steps 1 --warmup 0 --score-users 0 --hybrid-users 0 --c5-users 0 --tt-steps 0 --no-ingest --api-reps 0 --rank256-epochs 0 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -20 gpurun_out/bench_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_c4.json'));print(json.dumps(d['tt_item_vectors_c4']));print(json.dumps(d['tt_scoring_c4']))"
