#!/bin/bash
# Build an A/B variant of libtadpole_hip.so with extra -D flags on one source:
#   tools/build_variant.sh <tag> <source.hip> "-DFOO=0 -DBAR=1"
# -> tadpole_amd/libtadpole_hip_<tag>.so (load it with TADPOLE_LIB=...)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/tadpole_amd/csrc
tag=$1; src=$2; defs=$3
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result -I/opt/rocm/include -D__HIP_PLATFORM_AMD__"
base=$(basename "$src" .hip)
/opt/rocm/bin/hipcc $FLAGS $defs -c "$C/$src" -o "$C/build/${base}_$tag.o"
objs=""
for o in "$C"/build/*.o; do
  [ -f "$C/$(basename "$o" .o).hip" ] || continue   # other variants' objects
  [ "$(basename "$o" .o)" = "$base" ] && o="$C/build/${base}_$tag.o"
  objs="$objs $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/tadpole_amd/libtadpole_hip_$tag.so" $objs -ldl
echo "built tadpole_amd/libtadpole_hip_$tag.so"
