#!/bin/bash
# Copy split of the streamed single calls' slice packing: 1 / 2 / 4 / 8
# threads per copy (STORB_RS_FORCE_PARTS builds), pageable encode + decode.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3s; mkdir -p $O
for a in "4 6 1048576" "16 24 8388608" "32 48 33554432"; do
  for N in p1 p2 nt1 nt2; do
    for op in encode decode; do
      echo -n "$N $a: " >> $O/parts.txt
      LD_LIBRARY_PATH=tools/_build/$N timeout -k 10 60 ./tools/_build/callprobe $a 100 $op pageable >> $O/parts.txt 2>&1 || { echo "callprobe failed"; tail -3 $O/parts.txt; exit 1; }
    done
  done
done
cat $O/parts.txt
