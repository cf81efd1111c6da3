#!/bin/bash
# k = 16 download mixed launch cap A/B (rs_device.hpp mix_ks_cap): the in-tree
# build against experiment builds, config 5 with download patterns.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r6s_abmix16; rm -rf $out; mkdir -p $out
export TMPDIR=/tmp
libs="storb_amd/lib/libstorb_rs.so $(ls storb_amd/lib/variants/*.so)"
for r in 1 2 3; do
  for lib in $libs; do
    tag=$(basename $lib .so)
    timeout -k 10 120 python tools/lib_ab.py $lib --config 5 --steps 100 --warmup 10 --minimal \
      --erase-pattern download > $out/${tag}_$r.json 2>> $out/err.log || exit $?
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['leg_ms'])" $out/${tag}_$r.json
  done
done
