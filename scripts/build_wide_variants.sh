# Timing-only builds of libhrec with HREC_WIDE_CUT=1 (Gramian only) and 2
# (no substitutions) -> hybrid-als-twotower-recommender_amd/lib/ab/
set -e
L=hybrid-als-twotower-recommender_amd/lib
mkdir -p $L/variants
for c in 1 2; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DHREC_WIDE_CUT=$c -c hybrid-als-twotower-recommender_amd/csrc/als_wide.hip -o /tmp/als_wide_cut$c.o
  objs=$(ls $L/obj/*.o | grep -v als_wide)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs /tmp/als_wide_cut$c.o -o $L/variants/libhrec_cut$c.so
done
