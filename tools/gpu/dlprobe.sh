#!/bin/bash
# HBM ceiling of the download decode's access shape (tools/dlprobe.hip).
# usage (via gpurun): bash tools/gpu/dlprobe.sh OUTDIR [rounds] [reps] [k4|k16|k32]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}
mkdir -p "$out"
make -s -C tools dlprobe > "$out/build.log" 2>&1 || { tail "$out/build.log"; exit 1; }
timeout -k 10 300 tools/_build/dlprobe "${2:-7}" "${3:-8}" ${4:-} > "$out/dlprobe.txt" 2>&1 || exit $?
cat "$out/dlprobe.txt"
