# A/B of the GEMV (csrc/dot_gemv.hip) build knobs on the c4 B = 1 call.
set -e
mkdir -p gpurun_out
V=hybrid-als-twotower-recommender_amd/lib/variants
for r in 1 2; do
  for n in ${GEMV_VARIANTS:-base}; do
    lib=$V/libhrec_gemv_$n.so; [ "$n" = base ] && lib=hybrid-als-twotower-recommender_amd/lib/libhrec.so
    echo "== $n"; HREC_LIB=$lib timeout -k 10 200 python -u scripts/gemv_probe.py 2>&1 | grep -v amdgpu.ids
  done
done
echo "== MFMA path (HREC_DOT_GEMV=0)"; HREC_DOT_GEMV=0 timeout -k 10 200 python -u scripts/gemv_probe.py 2>&1 | grep -v amdgpu.ids
