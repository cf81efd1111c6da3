#!/bin/bash
# <8,3> launch shape A/B (rs_device.hpp PermShape<8,3>) on bench --config 3:
# the in-tree build against experiment builds, interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r6s_ab83; rm -rf $out; mkdir -p $out
export TMPDIR=/tmp
libs="storb_amd/lib/libstorb_rs.so $(ls storb_amd/lib/variants/*.so)"
for r in 1 2 3; do
  for lib in $libs; do
    tag=$(basename $lib .so)
    timeout -k 10 120 python tools/lib_ab.py $lib --config 3 --steps 200 --warmup 10 --minimal \
      > $out/${tag}_$r.json 2>> $out/err.log || exit $?
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['leg_ms'])" $out/${tag}_$r.json
  done
done
