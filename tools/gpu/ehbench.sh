#!/bin/bash
# Chunk-phase shapes of the encode + piece-id kernel (tools/ehbench.hip),
# then one PMC pass (VALU issue, waits) over a single launch of each.
# usage: tools/gpu/ehbench.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
# tools/_build does not travel to the box (.gpurunignore): build there
make -s -j4 -C tools ehbench > /dev/null || exit 1
O=gpurun_out/${1:-eh}; mkdir -p $O
timeout -k 10 240 tools/_build/ehbench 5 5 > $O/ehbench.txt 2>&1 || { cat $O/ehbench.txt; exit 1; }
cat $O/ehbench.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVES --output-format csv -d "$GRAFT_REPO_ROOT/$O/pmc" -o run -- "$GRAFT_REPO_ROOT/tools/_build/ehbench" 1 1 > "$GRAFT_REPO_ROOT/$O/pmc.log" 2>&1 || { tail "$GRAFT_REPO_ROOT/$O/pmc.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
d=$(dirname $(find $O/pmc -name 'run_counter_collection.csv' | head -1))
python3 tools/valu_busy.py $d > $O/valu_busy.json 2>&1; cat $O/valu_busy.json
