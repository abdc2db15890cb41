set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_core.py tests/test_gpu_api.py tests/test_gpu_dot.py -x -q --timeout 120 --timeout-method thread -k "hybrid or fusion or tt or twotower or score" > gpurun_out/v2_tests.log 2>&1 || { tail -30 gpurun_out/v2_tests.log; exit 1; }
tail -1 gpurun_out/v2_tests.log
for r in 1 2; do for n in v1 v2; do echo -n "$n "; HREC_LIB=hybrid-als-twotower-recommender_amd/lib/ab/libhrec_$n.so timeout -k 5 60 python scripts/tt_score_quick.py 2>&1 | grep tt_score; done; done
bash scripts/ab_hybrid.sh
