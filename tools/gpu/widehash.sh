#!/bin/bash
# Wide-geometry encode + piece ids: the pipelining settings timed, then one
# rocprofv3 kernel trace of the sequential and the best-guess setting.
# usage (via gpurun): bash tools/gpu/widehash.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python tools/widehash.py > "$out/widehash.jsonl" 2> "$out/widehash.err" || exit $?
cat "$out/widehash.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
  python3 tools/widehash.py --reps 5 > "$out/prof.jsonl" 2>> "$out/widehash.err" || exit $?
