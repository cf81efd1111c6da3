#!/bin/bash
# Batch host paths (tools/hostpath.py, 12 reps) by host copy threads.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/hostthreads; mkdir -p $out
for r in 1 2 3; do
  for t in 4 8; do
    for zc in 1 0; do
      STORB_RS_ZC_BATCH=$zc STORB_RS_HOST_THREADS=$t timeout -k 10 200 python tools/hostpath.py --reps 12 >> $out/hostpath.jsonl 2>> $out/err.log || exit $?
      tail -1 $out/hostpath.jsonl | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['env'], d['value'], d['pinned_value'], d['hashed_value'], d['decode_value'], d['decode_pinned_value'], d['decode_download_value'])"
    done
  done
done
