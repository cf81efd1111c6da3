#!/bin/bash
# The -m gpu suite, smoke() and the default bench line (with the kernel-trace
# passes), plus the clock / GRBM probe.  usage (via gpurun): bash tools/gpu/r5_check.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}
mkdir -p "$out"
export TMPDIR=/tmp
bash tools/gpu/clocks.sh "$out/clk" || exit $?
t0=$(date +%s.%N)
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" || exit $?
t1=$(date +%s.%N)
echo "bench wall $(python3 -c "print(round($t1-$t0,1))") s"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/gputest.log" 2>&1
rc=$?
tail -2 "$out/gputest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.log" 2>&1 || exit $?
tail -1 "$out/smoke.log"
