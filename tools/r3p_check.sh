#!/bin/bash
# Streamed bit-sliced encodes ((16,24), (32,48)) + the earlier streamed
# calls: parity tests, fuzz, latency; JIT compile progress in a torch
# process; the (8, 12) 4 MiB single-call anomaly traced.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3p; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_piece_api.py tests/test_gpu_async.py tests/test_gpu_runtime.py tests/test_gpu_patterns.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/fuzz.py --seconds 60 --seed 47 > $O/fuzz.json 2>&1 || { echo "fuzz failed"; tail -20 $O/fuzz.json; exit 1; }
tail -1 $O/fuzz.json
for a in "16 24 8388608" "32 48 33554432" "8 12 4194304"; do
  for op in encode decode; do
    for m in pageable pinned; do
      timeout -k 10 60 ./tools/_build/callprobe $a 100 $op $m >> $O/callprobe.jsonl 2>&1 || { echo "callprobe $a $op $m failed"; tail -3 $O/callprobe.jsonl; exit 1; }
    done
  done
done
cat $O/callprobe.jsonl
for a in "8 12 4194304" "16 24 8388608"; do
  echo "== $a encode pageable" >> $O/calltrace.txt
  LD_LIBRARY_PATH=tools/_build/tr timeout -k 10 60 ./tools/_build/callprobe_trace $a 100 encode pageable >> $O/calltrace.txt 2>&1 || { echo "trace failed"; tail -3 $O/calltrace.txt; exit 1; }
done
cat $O/calltrace.txt
i=0
for m in idle torch decode; do
  i=$((i+1))
  timeout -k 10 90 python -u tools/jit_contend.py $m $((i*37+5)) >> $O/jit_contend_py.txt 2>&1 || { echo "jit_contend $m failed"; tail -5 $O/jit_contend_py.txt; exit 1; }
done
grep -v amdgpu.ids $O/jit_contend_py.txt
