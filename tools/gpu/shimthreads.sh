#!/bin/bash
# Per-chunk drop-in call latency by host copy threads (tools/shimpath.py).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/shimthreads; mkdir -p $out
for r in 1 2; do
  for t in 4 8 12 16; do
    STORB_RS_HOST_THREADS=$t timeout -k 10 200 python tools/shimpath.py >> $out/shim.jsonl 2>> $out/err.log || exit $?
    tail -1 $out/shim.jsonl
  done
done
