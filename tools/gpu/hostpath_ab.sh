#!/bin/bash
# Batch host paths (tools/hostpath.py, 12 reps per figure), library builds
# interleaved, SDMA forced (STORB_RS_ZC_BATCH=0) and default.
# usage (via gpurun): bash tools/gpu/hostpath_ab.sh OUTDIR ROUNDS LIB...
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}; rounds=${2:?rounds}; shift 2
mkdir -p $out
for r in $(seq $rounds); do
  for lib in "$@"; do
    for zc in 1 0; do
      STORB_RS_ZC_BATCH=$zc timeout -k 10 200 python tools/hostpath.py --reps 12 --lib $lib >> $out/hostpath.jsonl 2>> $out/err.log || exit $?
      tail -1 $out/hostpath.jsonl | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['lib'].split('/')[-2], d['env']['STORB_RS_ZC_BATCH'], d['value'], d['pinned_value'], d['hashed_value'], d['decode_value'], d['decode_pinned_value'], d['decode_download_value'])"
    done
  done
done
