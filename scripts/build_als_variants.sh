# Build A/B variants of libhrec that differ only in csrc/als.hip's defines:
# the other objects are reused from lib/obj (run build() first).
# usage: bash scripts/build_als_variants.sh "NAME:-DFLAG=1 -DOTHER=2" ...
set -e
D=hybrid-als-twotower-recommender_amd
mkdir -p $D/lib/ab
OBJS=$(ls $D/lib/obj/*.o | grep -v '/als.hip.o$')
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  (
    timeout -k 5 900 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result \
      $flags -c $D/csrc/als.hip -o $D/lib/ab/als_$name.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS $D/lib/ab/als_$name.o -o $D/lib/ab/libhrec_$name.so &&
    rm -f $D/lib/ab/als_$name.o
  ) &
done
wait
ls -la $D/lib/ab
