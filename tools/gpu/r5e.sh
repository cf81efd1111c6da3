#!/bin/bash
# Download-decode ceiling probe, config-5 loopback at 1 GiB, default bench line.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5e
mkdir -p $out
export TMPDIR=/tmp
bash tools/gpu/dlprobe.sh $out 7 8 || exit $?
timeout -k 10 300 python tools/loopback.py > $out/loopback.json 2> $out/loopback.err || exit $?
cat $out/loopback.json
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || exit $?
echo bench ok
