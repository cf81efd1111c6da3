#!/bin/bash
# Mixed-row descriptor decode at k = 32 (config 6 download shape): cap / tpw sweep.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3za; mkdir -p $O
timeout -k 10 120 tools/_build/descbench 30 32 > $O/descbench32.txt 2>&1 && cat $O/descbench32.txt &&
timeout -k 10 120 tools/_build/descbench 30 16 > $O/descbench16.txt 2>&1 && cat $O/descbench16.txt
