#!/bin/bash
# Streamed single calls (one launch per call gated on host-written slice
# words): parity tests, differential fuzz, latency; JIT compile progress
# with the GPU idle vs busy.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3o; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_piece_api.py tests/test_gpu_async.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/fuzz.py --seconds 90 --seed 31 > $O/fuzz.json 2>&1 || { echo "fuzz failed"; tail -20 $O/fuzz.json; exit 1; }
tail -2 $O/fuzz.json
for a in "2 3 262144" "4 6 1048576" "8 12 4194304" "16 24 8388608"; do
  for op in encode decode; do
    for m in pageable pinned; do
      timeout -k 10 60 ./tools/_build/callprobe $a 400 $op $m >> $O/callprobe.jsonl 2>&1 || { echo "callprobe $a $op $m failed"; tail -3 $O/callprobe.jsonl; exit 1; }
    done
  done
done
cat $O/callprobe.jsonl
for a in "4 6 1048576" "2 3 262144"; do
  for op in encode decode; do
    echo "== $a $op pageable" >> $O/calltrace.txt
    LD_LIBRARY_PATH=tools/_build/tr timeout -k 10 60 ./tools/_build/callprobe_trace $a 300 $op pageable >> $O/calltrace.txt 2>&1 || { echo "trace failed"; tail -3 $O/calltrace.txt; exit 1; }
  done
done
cat $O/calltrace.txt
timeout -k 10 60 ./tools/_build/jit_contend idle 11 > $O/jit_contend.txt 2>&1 || { echo "jit_contend failed"; tail $O/jit_contend.txt; exit 1; }
timeout -k 10 60 ./tools/_build/jit_contend gpu 23 >> $O/jit_contend.txt 2>&1 || { echo "jit_contend failed"; tail $O/jit_contend.txt; exit 1; }
cat $O/jit_contend.txt
