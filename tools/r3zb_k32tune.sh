#!/bin/bash
# Launch-shape sweep of the table kernel at k = 32 (tools/k32_tune.hip).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3zb; mkdir -p $O
timeout -k 10 240 tools/_build/k32_tune 25 > $O/k32_tune.txt 2>&1; rc=$?
cat $O/k32_tune.txt; exit $rc
