#!/bin/bash
# Round check on the current tree: GPU suite, smoke, the default bench line
# (the driver's command), and the download timeline.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5n; mkdir -p $out
export TMPDIR=/tmp
bash tools/gpu/dltrace.sh $out/dl > $out/dltrace.txt 2>&1 || exit $?
head -12 $out/dltrace.txt
t0=$(date +%s.%N)
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || exit $?
t1=$(date +%s.%N)
echo "bench wall $(python3 -c "print(round($t1-$t0,1))") s"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/gputest.log 2>&1 || { tail -30 $out/gputest.log; exit 1; }
tail -2 $out/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log
