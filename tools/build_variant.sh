#!/bin/bash
# An experiment build of the library: one kernel translation unit recompiled
# with extra -D flags, linked with the in-tree objects of the others.
# usage: bash tools/build_variant.sh TAG TU.hip "-DFOO=1 ..."  ->  storb_amd/lib/variants/libstorb_rs_TAG.so
set -euo pipefail
cd "$(dirname "$0")/../storb_amd"
tag=$1; tu=$2; flags=$3
make -s -j16 >/dev/null
mkdir -p lib/variants build/variants
base=$(basename "$tu" .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $flags \
  -c "csrc/$tu" -o "build/variants/${base}_$tag.o"
objs=$(ls build/*.o | grep -v "/$base.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o "lib/variants/libstorb_rs_$tag.so" \
  $objs "build/variants/${base}_$tag.o" -lhiprtc -lamd_comgr -Wl,-soname,libstorb_rs.so
echo "lib/variants/libstorb_rs_$tag.so"
