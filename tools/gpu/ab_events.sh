#!/bin/bash
# Interleaved A/B of library builds on the headline step and config 2's download
# step (round 5: the per-launch order events against sparse marks).
# usage (via gpurun): bash tools/gpu/ab_events.sh OUTDIR ROUNDS LIB...
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}; rounds=${2:?rounds}; shift 2
libs=("$@")
mkdir -p $out
export TMPDIR=/tmp
for r in $(seq $rounds); do
  for lib in "${libs[@]}"; do
    tag=$(basename $(dirname $lib))
    for mode in fixed download; do
      timeout -k 10 120 python tools/lib_ab.py $lib --steps 400 --warmup 10 --erase-pattern $mode \
        --minimal > $out/${mode}_${tag}_$r.json 2>> $out/err.log || exit $?
      python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[2], sys.argv[3], d['value'], r['gpu_ms_per_step'], r['leg_ms'])" $out/${mode}_${tag}_$r.json $mode $tag
    done
  done
done
