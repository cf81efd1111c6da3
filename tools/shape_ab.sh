#!/bin/bash
# Launch-shape A/B of the run-time-compiled bit-sliced decode on the real
# bench decode path: STORB_RS_JIT_SHAPE="threads,swz,cap" per run (rs_jit.cpp
# shape()), STORB_RS_JIT=always so every decode runs compiled. One bench line
# per (case, shape) in gpurun_out/ab_<case>_<shape>.log.
# usage: bash tools/shape_ab.sh "c5e8 c6e16" "64,1,6 128,0,4 256,1,2"
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
CASES=${1:-"c5e8"}
SHAPES=${2:-"default"}
for c in $CASES; do
  case $c in
    c3) args="--config 3" ;;
    c5e*) args="--config 5 --erase ${c#c5e}" ;;
    c6e*) args="--config 6 --erase ${c#c6e}" ;;
  esac
  for sh in $SHAPES; do
    if [ "$sh" = default ]; then unset STORB_RS_JIT_SHAPE; else export STORB_RS_JIT_SHAPE=$sh; fi
    STORB_RS_JIT=always timeout -k 10 200 python3 bench.py $args --cpu-seconds 0 --no-host-path \
      --no-traffic > "gpurun_out/ab_${c}_${sh//,/_}.log" 2>&1
    echo "$c $sh done"
  done
done
unset STORB_RS_JIT_SHAPE
