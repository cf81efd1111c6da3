#!/bin/bash
# Pattern / parity GPU tests, then the default bench line (the driver's
# command): download leg with its settle pre-roll and host cost per call.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5z; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_patterns.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['frac']); dd=d['download_decode']
print({k: dd.get(k) for k in ('ms_per_call','host_us_per_call','settle')}, dd['roofline']['frac'], dd.get('kernel_trace',{}).get('avg_us'), dd.get('kernel_trace',{}).get('call_overhead_us'))"
