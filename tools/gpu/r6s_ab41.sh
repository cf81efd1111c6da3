#!/bin/bash
# <4,1> launch shape A/B (rs_device.hpp PermShape<4,1>) on the default line's
# repair leg (one share rebuilt per stripe from 4, in place): the in-tree
# build against experiment builds, interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r6s_ab41; rm -rf $out; mkdir -p $out
export TMPDIR=/tmp
libs="storb_amd/lib/libstorb_rs.so $(ls storb_amd/lib/variants/*.so)"
for r in 1 2 3; do
  for lib in $libs; do
    tag=$(basename $lib .so)
    timeout -k 10 120 python tools/lib_ab.py $lib --steps 20 --warmup 5 --cpu-seconds 0 --no-host-path --no-traffic \
      > $out/${tag}_$r.json 2>> $out/err.log || exit $?
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['repair'];print(sys.argv[1], d['value'], r['data']['ms'], r['parity']['ms'])" $out/${tag}_$r.json
  done
done
