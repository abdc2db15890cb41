# K1w (ranks 65..256): parity tests, then the rank-256 timing probe, A/B
# against the variant libraries in lib/abw (if present)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_als_wide.py -q -x --timeout 240 --timeout-method thread > gpurun_out/wide_tests.log 2>&1 || { tail -30 gpurun_out/wide_tests.log; exit 1; }
tail -1 gpurun_out/wide_tests.log
for r in 1 2; do
  for lib in hybrid-als-twotower-recommender_amd/lib/abw/*.so; do echo -n "$(basename $lib): "; HREC_LIB=$lib timeout -k 10 200 python scripts/wide_quick.py 256 300000 100000; done
  echo -n "head: "; timeout -k 10 200 python scripts/wide_quick.py 256 300000 100000
done
# bit-identity of the variants (rank 256 and 128 factors after 2 epochs)
for k in 256 128; do
  for lib in hybrid-als-twotower-recommender_amd/lib/abw/*.so; do HREC_LIB=$lib timeout -k 10 120 python scripts/als_checksum.py $k; done
  timeout -k 10 120 python scripts/als_checksum.py $k
done
# parity of each variant library (the wide tests through HREC_LIB)
for lib in hybrid-als-twotower-recommender_amd/lib/abw/*.so; do HREC_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_als_wide.py -q -x --timeout 240 --timeout-method thread 2>&1 | tail -1; done
