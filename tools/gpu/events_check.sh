#!/bin/bash
# After a runtime change: the GPU modules that exercise it, then three default
# bench lines (value, leg times, CPU baseline diagnostics).
# usage: tools/gpu/events_check.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-ev}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_lifetime.py tests/test_gpu_patterns.py tests/test_gpu_jit.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-host-path --no-traffic > $O/bench$i.json 2> $O/bench$i.err || { tail $O/bench$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench$i.json').read().strip().splitlines()[-1]); r=d['roofline']; c=d['cpu_baseline']
print('bench', d['value'], r['frac'], r['leg_ms'], r['gpu_ms_per_step'])
print('cpu', c['value'], c['arithmetic_only']['value'], json.dumps(c['thread']))"
done
