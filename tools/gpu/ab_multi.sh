#!/bin/bash
# Interleaved A/B of several library builds on the download legs (configs 2
# and 5, --erase-pattern download), after the pattern tests on the last one.
# usage (via gpurun): bash tools/gpu/ab_multi.sh OUTDIR ROUNDS LIB...
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}; rounds=${2:?rounds}; shift 2
libs=("$@")
mkdir -p $out
export TMPDIR=/tmp
# (the tests load the in-tree build)
timeout -k 10 400 python -u -m pytest tests/test_gpu_patterns.py tests/test_gpu_dist.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in $(seq $rounds); do
  for lib in "${libs[@]}"; do
    tag=$(basename $(dirname $lib))
    for c in ${CFGS:-"2:200 5:100"}; do
      cfg=${c%:*}; steps=${c#*:}
      timeout -k 10 120 python tools/lib_ab.py $lib --config $cfg --steps $steps --warmup 10 --erase-pattern download \
        --minimal > $out/c${cfg}_${tag}_$r.json 2>> $out/err.log || exit $?
      python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], sys.argv[3], d['value'], d['roofline']['leg_ms'])" $out/c${cfg}_${tag}_$r.json c$cfg $tag
    done
  done
done
