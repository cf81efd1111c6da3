#!/bin/bash
# Interleaved A/B of library builds on the headline workloads (config 2,
# config 4's 10,000-object launch).  usage: bash tools/gpu/ab_headline.sh OUTDIR ROUNDS LIB...
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}; rounds=${2:?rounds}; shift 2
libs=("$@")
mkdir -p $out
export TMPDIR=/tmp
for r in $(seq $rounds); do
  for lib in "${libs[@]}"; do
    tag=$(basename $(dirname $lib))
    for c in "2 200" "4 20"; do
      cfg=${c% *}; steps=${c#* }
      timeout -k 10 180 python tools/lib_ab.py $lib --config $cfg --steps $steps --warmup 10 \
        --minimal > $out/c${cfg}_${tag}_$r.json 2>> $out/err.log || exit $?
      python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], sys.argv[3], d['value'], d['roofline']['gpu_ms_per_step'], d['roofline']['leg_ms'])" $out/c${cfg}_${tag}_$r.json c$cfg $tag
    done
  done
done
