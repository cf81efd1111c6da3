#!/bin/bash
# H2D / D2H overlap by stream arrangement (tools/sdma_probe.hip).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}; mkdir -p $out
make -s -C tools sdma_probe > $out/build.log 2>&1 || { tail $out/build.log; exit 1; }
timeout -k 10 200 tools/_build/sdma_probe 5 > $out/sdma.txt 2>&1 || { cat $out/sdma.txt; exit 1; }
cat $out/sdma.txt
