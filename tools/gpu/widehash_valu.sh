#!/bin/bash
# SQ counters (VALU issue, waits) of the wide-geometry encode and hash kernels
# (tools/widehash.py, sequential setting only), summarised by tools/valu_busy.py.
# usage (via gpurun): bash tools/gpu/widehash_valu.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${1:?outdir}; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVES --output-format csv -d "$R/$O/pmc" -o run -- python3 "$R/tools/widehash.py" --reps 2 > "$R/$O/pmc.log" 2>&1 || { tail "$R/$O/pmc.log"; exit 1; }
cd "$R"
d=$(dirname $(find $O/pmc -name 'run_counter_collection.csv' | head -1))
python3 tools/valu_busy.py $d > $O/valu_busy.json 2>&1; cat $O/valu_busy.json
