#!/bin/bash
# Host-path settings A/B (one process per setting), the differential fuzz on
# the round's code, and the newest GPU tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5o; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_blake3.py -m gpu -x -q -k pitched --timeout 120 \
  --timeout-method thread > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for env in "" "STORB_RS_ZC_BATCH=0" "STORB_RS_HOST_THREADS=16" "STORB_RS_ZC_BATCH=0 STORB_RS_HOST_THREADS=16"; do
    env $env timeout -k 10 200 python tools/hostpath.py >> $out/hostpath.jsonl 2>> $out/err.log || exit $?
    tail -1 $out/hostpath.jsonl | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['env'], d['value'], d['pinned_value'], d['hashed_value'], d['decode_value'], d['decode_pinned_value'], d['decode_download_value'], d['pcie']['both_GBps'])"
  done
done
timeout -k 10 200 python tools/fuzz.py --seconds 120 --seed 5005 > $out/fuzz.json 2> $out/fuzz.err || { tail -5 $out/fuzz.err; exit 1; }
cat $out/fuzz.json
