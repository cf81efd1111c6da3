#!/bin/bash
# Per-direction staging streams: hostpath.py old/new interleaved, 12 reps per
# figure, SDMA forced (STORB_RS_ZC_BATCH=0), 8 and 16 host copy threads.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5y; mkdir -p $out
export TMPDIR=/tmp
for r in 1 2 3 4; do
  for lib in storb_amd/lib/ab_old/libstorb_rs.so storb_amd/lib/libstorb_rs.so; do
    for env in "STORB_RS_ZC_BATCH=0 STORB_RS_HOST_THREADS=8" "STORB_RS_ZC_BATCH=0 STORB_RS_HOST_THREADS=16"; do
      env $env timeout -k 10 200 python tools/hostpath.py --reps 12 --lib $lib >> $out/hostpath.jsonl 2>> $out/err.log || exit $?
      tail -1 $out/hostpath.jsonl | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['lib'].split('/')[-2], d['env']['STORB_RS_HOST_THREADS'], d['value'], d['pinned_value'], d['hashed_value'], d['decode_value'], d['decode_pinned_value'], d['decode_download_value'], d['pcie']['both_GBps'])"
    done
  done
done
