#!/bin/bash
# Mixed-row descriptor decode kernel variants (tools/mixbench.hip), k = 16 and 32.
# usage: tools/gpu/mixbench.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
# tools/_build does not travel to the box (.gpurunignore): build there
make -s -j4 -C tools mixbench > /dev/null || exit 1
O=gpurun_out/${1:-mix}; mkdir -p $O
timeout -k 10 180 tools/_build/mixbench 25 16 > $O/mixbench16.txt 2>&1 && cat $O/mixbench16.txt &&
timeout -k 10 180 tools/_build/mixbench 25 32 > $O/mixbench32.txt 2>&1; rc=$?
cat $O/mixbench32.txt; exit $rc
