# One-file A/B variant of libhrec: rebuild FILE.hip with extra FLAGS and link it
# with the main build's other objects (lib/obj) into lib/v6/libhrec_NAME.so.
#   bash scripts/build_variant_obj.sh NAME "FLAGS" file.hip [file2.hip ...]
set -e
D=hybrid-als-twotower-recommender_amd
name=$1; flags=$2; shift 2
python -c "import __graft_entry__ as g; g.build_lib()"
mkdir -p $D/lib/v6/$name
objs=""
for o in $D/lib/obj/*.o; do
  base=$(basename $o .o)
  skip=0
  for f in "$@"; do [ "$base" = "$f" ] && skip=1; done
  [ $skip = 0 ] && objs="$objs $o"
done
for f in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $flags -c $D/csrc/$f -o $D/lib/v6/$name/$f.o
  objs="$objs $D/lib/v6/$name/$f.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o $D/lib/v6/libhrec_$name.so
rm -rf $D/lib/v6/$name
echo built $D/lib/v6/libhrec_$name.so
