#!/bin/bash
# Single-call latency anatomy (storb_rs_encode / _decode, Storb's sizing of
# 1 MiB and 16 MiB objects): plain timings, then a runtime + kernel trace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3i; mkdir -p $O
for a in "2 3 262144" "4 6 1048576" "16 24 8388608"; do
  for op in encode decode; do
    for m in pageable pinned; do
      timeout -k 10 60 ./tools/_build/callprobe $a 400 $op $m >> $O/callprobe.jsonl 2>&1 || { echo "callprobe $a $op $m failed"; tail -3 $O/callprobe.jsonl; exit 1; }
    done
  done
done
cat $O/callprobe.jsonl
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/trace_enc46 -o run -- ./tools/_build/callprobe 4 6 1048576 200 encode pageable > $O/trace_enc46.log 2>&1 || { echo "trace failed"; tail -5 $O/trace_enc46.log; exit 1; }
echo traced
