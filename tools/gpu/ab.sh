#!/bin/bash
# A/B of two library builds on the download legs (tools/lib_ab.py), after the
# pattern tests on the new build.  usage (via gpurun): bash tools/gpu/ab.sh OUTDIR BASELIB
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}; base=${2:?base lib}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_patterns.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2; do
  for lib in $base storb_amd/lib/libstorb_rs.so; do
    tag=$(echo $lib | tr '/' '_')
    for c in "2 200" "5 100"; do
      set -- $c
      timeout -k 10 120 python tools/lib_ab.py $lib --config $1 --steps $2 --warmup 10 --erase-pattern download \
        --minimal > $out/c$1_${tag}_$r.json 2>> $out/err.log || exit $?
      python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1], d['value'], d['roofline']['leg_ms'])" $out/c$1_${tag}_$r.json
    done
  done
done
