mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_dot.py -k "prune or bf16_paths or unknown_rows" -v --timeout 120 --timeout-method thread > gpurun_out/prune.log 2>&1; tail -15 gpurun_out/prune.log
timeout -k 10 300 python -u scripts/trained_ranking_diag.py > gpurun_out/diag.log 2>&1; cat gpurun_out/diag.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_api.py -k "numpy_fusion or device_path or end_to_end" -q --timeout 120 --timeout-method thread > gpurun_out/api.log 2>&1; tail -3 gpurun_out/api.log
