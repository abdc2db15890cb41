# Build A/B variants of libhrec into hybrid-als-twotower-recommender_amd/lib/ab/
# usage: bash scripts/build_variants.sh "NAME:-DFLAG=1 -DOTHER=2" ...
set -e
D=hybrid-als-twotower-recommender_amd
mkdir -p $D/lib/ab
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  timeout -k 5 900 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $flags $D/csrc/*.hip -o $D/lib/ab/libhrec_$name.so &
done
wait
ls -la $D/lib/ab
