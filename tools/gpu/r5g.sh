#!/bin/bash
# Sparse order marks (ctx.hpp StreamMarks): the GPU suite on the new build,
# a fuzz, then the old / new A/B on the headline and download steps.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5g; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread \
  > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 200 python tools/fuzz.py --seconds 100 --seed 7404 > $out/fuzz.json 2> $out/fuzz.err || { tail -5 $out/fuzz.err; exit 1; }
tail -1 $out/fuzz.json
bash tools/gpu/ab_events.sh $out 3 storb_amd/lib/ab_old/libstorb_rs.so storb_amd/lib/libstorb_rs.so
