#!/bin/bash
# <2,1> launch shape A/B on Storb's (2, 3) encode and in-place decode (tools/ab21.py).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r6s_ab21; rm -rf $out; mkdir -p $out
libs="storb_amd/lib/libstorb_rs.so $(ls storb_amd/lib/variants/*.so)"
for r in 1 2 3; do
  for lib in $libs; do
    tag=$(basename $lib .so)
    timeout -k 10 120 python tools/ab21.py $lib > $out/${tag}_$r.json 2>> $out/err.log || exit $?
    echo "$tag $(cat $out/${tag}_$r.json)"
  done
done
