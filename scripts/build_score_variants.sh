# score.hip A/B variants linked with the library's other objects
# usage: bash scripts/build_score_variants.sh "NAME:-DFLAG=1" ...
set -e
D=hybrid-als-twotower-recommender_amd
mkdir -p $D/lib/variants /tmp/scvar
objs=$(ls $D/lib/obj/*.o | grep -v score.hip.o)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $flags -c $D/csrc/score.hip -o /tmp/scvar/score_$name.o && \
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC /tmp/scvar/score_$name.o $objs -o $D/lib/variants/libhrec_$name.so ) &
done
wait
ls $D/lib/variants
