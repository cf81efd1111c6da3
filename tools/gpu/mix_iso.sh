#!/bin/bash
# mixbench (variants + per-row-count isolation) and a rocprof of descbench's
# config 6 download shape (the uniform rs_apply_perm<32,2> and the product path).
# usage: tools/gpu/mix_iso.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-mixiso}; mkdir -p $O
timeout -k 10 180 tools/_build/mixbench 25 16 > $O/mixbench16.txt 2>&1 && cat $O/mixbench16.txt &&
timeout -k 10 180 tools/_build/mixbench 25 32 > $O/mixbench32.txt 2>&1 && cat $O/mixbench32.txt || exit 1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_desc32 -o run -- tools/_build/descbench 20 32 > $O/descbench32_traced.txt 2>&1 || exit 1
find $O/trace_desc32 -name "*kernel_trace.csv" -delete
cat $O/descbench32_traced.txt
grep -h "rs_apply" $(find $O/trace_desc32 -name "*kernel_stats.csv") | cut -c1-200
