#!/bin/bash
# Final tree: the streamed-slices test and wide-decode latency, then the
# driver's round-end sequence.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3x; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "streamed or large_ragged or single_call" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for a in "16 24 8388608" "32 48 33554432"; do
  timeout -k 10 60 ./tools/_build/callprobe $a 100 decode pageable >> $O/callprobe.jsonl 2>&1 || { echo "callprobe failed"; exit 1; }
done
cat $O/callprobe.jsonl
bash tools/round_check.sh || exit $?
