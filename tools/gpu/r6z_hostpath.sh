#!/bin/bash
# Host-inclusive decode timed as the C ABI is called (share pointers
# marshalled before the timed loop): hostpath at config 2 and 5 geometry,
# default library settings, after the decode_chunks GPU tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r6z; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_patterns.py -m gpu -x -q \
  -k "chunks" --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 150 python tools/fuzz.py --seconds ${FUZZ_S:-60} --seed 6107 > $out/fuzz.json 2> $out/fuzz.err || { tail -5 $out/fuzz.err; exit 1; }
tail -c 400 $out/fuzz.json; echo
for g in "4 6 1048576 256" "16 24 8388608 32"; do
  set -- $g
  for z in 1 0; do
    STORB_RS_ZC_BATCH=$z timeout -k 10 150 python tools/hostpath.py --k $1 --n $2 --chunk $3 --chunks $4 \
      > $out/hp_k$1_zc$z.json 2> $out/hp_k$1_zc$z.err || exit $?
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1], {k:v for k,v in d.items() if 'value' in k}, d['pin'].get('cpus'))" $out/hp_k$1_zc$z.json
  done
done
