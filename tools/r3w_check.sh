#!/bin/bash
# Streamed table kernel up to k = 32 (single-call decode of the wide
# geometries): parity tests + fuzz + latency, then the round-end sequence.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_piece_api.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u tools/fuzz.py --seconds 45 --seed 53 > $O/fuzz.json 2>&1 || { echo "fuzz failed"; tail -20 $O/fuzz.json; exit 1; }
tail -1 $O/fuzz.json
for a in "16 24 8388608" "32 48 33554432" "4 6 1048576"; do
  for op in decode encode; do
    timeout -k 10 60 ./tools/_build/callprobe $a 100 $op pageable >> $O/callprobe.jsonl 2>&1 || { echo "callprobe $a $op failed"; tail -3 $O/callprobe.jsonl; exit 1; }
  done
done
cat $O/callprobe.jsonl
bash tools/round_check.sh || exit $?
