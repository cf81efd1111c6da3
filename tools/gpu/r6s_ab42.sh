#!/bin/bash
# Headline RS(4,2) launch shape A/B (rs_device.hpp PermShape<4,2>): the
# in-tree build against experiment builds (tools/build_variant.sh), the
# default bench line (--minimal), interleaved rounds. Out: gpurun_out/r6s_ab42/
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r6s_ab42; rm -rf $out; mkdir -p $out
export TMPDIR=/tmp
libs="storb_amd/lib/libstorb_rs.so $(ls storb_amd/lib/variants/*.so)"
for r in 1 2 3; do
  for lib in $libs; do
    tag=$(basename $lib .so)
    timeout -k 10 120 python tools/lib_ab.py $lib --steps 200 --warmup 10 --minimal \
      > $out/${tag}_$r.json 2>> $out/err.log || exit $?
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['leg_ms'])" $out/${tag}_$r.json
  done
done
# config 4 (the same kernel over 10,000 objects), the in-tree build against t64c14
if [ -e storb_amd/lib/variants/libstorb_rs_t64c14.so ]; then
  for r in 1 2; do
    for lib in storb_amd/lib/libstorb_rs.so storb_amd/lib/variants/libstorb_rs_t64c14.so; do
      tag=$(basename $lib .so)
      timeout -k 10 180 python tools/lib_ab.py $lib --config 4 --steps 20 --warmup 3 --minimal \
        > $out/c4_${tag}_$r.json 2>> $out/err.log || exit $?
      python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['leg_ms'])" $out/c4_${tag}_$r.json
    done
  done
fi
