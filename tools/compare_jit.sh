#!/bin/bash
# A/B of the run-time-compiled bit-sliced decode against the table kernel
# around the policy threshold (rs_jit.cpp wanted()): STORB_RS_JIT=0 vs
# =always on config 3's RS(8,4) with 3 lost and on RS(16,8) / RS(32,16)
# decodes with E lost. Bench lines in gpurun_out/cmp_<case>_<mode>.log.
# usage: bash tools/compare_jit.sh "c3 c5e2 c5e3 c6e2 c6e3"
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
CASES=${1:-"c3 c5e2"}
for c in $CASES; do
  case $c in
    c3) args="--config 3" ;;
    c5e*) args="--config 5 --erase ${c#c5e}" ;;
    c6e*) args="--config 6 --erase ${c#c6e}" ;;
  esac
  for v in 0 always; do
    STORB_RS_JIT=$v timeout -k 10 200 python3 bench.py $args --cpu-seconds 0 --no-host-path \
      --no-traffic > gpurun_out/cmp_${c}_$v.log 2>&1
  done
done
echo done
