#!/bin/bash
# Per-chunk drop-in calls, two library builds interleaved (tools/shimpath.py).
# usage (via gpurun): bash tools/gpu/shim_ab.sh OUTDIR ROUNDS LIB...
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}; rounds=${2:?rounds}; shift 2
mkdir -p $out
for r in $(seq $rounds); do
  for lib in "$@"; do
    timeout -k 10 200 python tools/shimpath.py --lib $lib >> $out/shim.jsonl 2>> $out/err.log || exit $?
    tail -1 $out/shim.jsonl
  done
done
