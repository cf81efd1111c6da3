#!/bin/bash
# <8,1> / <8,2> launch shape A/B on Storb's (8, 12) in-place decodes (tools/ab21.py AB_K=8).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r6s_ab8r; rm -rf $out; mkdir -p $out
libs="storb_amd/lib/libstorb_rs.so $(ls storb_amd/lib/variants/*.so)"
for r in 1 2; do
  for lost in 1 2; do
    for lib in $libs; do
      tag=$(basename $lib .so)
      AB_K=8 AB_LOST=$lost timeout -k 10 120 python tools/ab21.py $lib > $out/${tag}_l${lost}_$r.json 2>> $out/err.log || exit $?
      echo "$tag lost=$lost $(cat $out/${tag}_l${lost}_$r.json)"
    done
  done
done
