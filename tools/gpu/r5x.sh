#!/bin/bash
# Per-direction staging streams (host_batch.cpp Staging): the host-path GPU
# tests on the new build, then hostpath.py interleaved old/new, then a fuzz.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5x; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_blake3.py tests/test_gpu_patterns.py \
  tests/test_gpu_runtime.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 \
  || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for r in 1 2 3; do
  for lib in storb_amd/lib/ab_old/libstorb_rs.so storb_amd/lib/libstorb_rs.so; do
    for env in "STORB_RS_HOST_THREADS=8" "STORB_RS_ZC_BATCH=0 STORB_RS_HOST_THREADS=8"; do
      env $env timeout -k 10 200 python tools/hostpath.py --lib $lib >> $out/hostpath.jsonl 2>> $out/err.log || exit $?
      tail -1 $out/hostpath.jsonl | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['lib'].split('/')[-2], d['env']['STORB_RS_ZC_BATCH'], d['value'], d['pinned_value'], d['hashed_value'], d['decode_value'], d['decode_pinned_value'], d['decode_download_value'], d['pcie']['both_GBps'])"
    done
  done
done
timeout -k 10 200 python tools/fuzz.py --seconds 90 --seed 7303 > $out/fuzz.json 2> $out/fuzz.err || { tail -5 $out/fuzz.err; exit 1; }
cat $out/fuzz.json
