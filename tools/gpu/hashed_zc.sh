#!/bin/bash
# The hashed batch path from page-locked chunks: zero-copy fused kernel
# (default) against the staged pipeline (STORB_RS_ZC_BATCH=0), after the
# blake3 / fused-kernel GPU tests.
# usage: tools/gpu/hashed_zc.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-hzc}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_blake3.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for zc in 1 0 1b; do
  export STORB_RS_ZC_BATCH=${zc:0:1}
  timeout -k 10 300 python bench.py --no-traffic --cpu-seconds 0 > $O/bench_$zc.json 2> $O/bench_$zc.err || { tail $O/bench_$zc.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$zc.json').read().strip().splitlines()[-1])
p=d.get('pcie_inclusive') or {}
print('zc_batch $zc', {k:v for k,v in p.items() if k.endswith('value')})"
done
timeout -k 10 200 python tools/fuzz.py --seconds 120 > $O/fuzz.jsonl 2>&1 || { tail -20 $O/fuzz.jsonl; exit 1; }
tail -1 $O/fuzz.jsonl
