#!/bin/bash
# Descriptor decode after the address-space fix (global loads, s_load
# records, tables not hoisted across tiles): descbench, pattern tests,
# download-pattern bench legs for configs 5, 6, 2.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3h; mkdir -p $O
timeout -k 10 120 ./tools/_build/descbench 20 > $O/descbench.txt 2>&1 || { echo "descbench failed"; tail $O/descbench.txt; exit 1; }
cat $O/descbench.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_patterns.py tests/test_gpu_async.py tests/test_gpu_jit.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in "5" "6" "2"; do
  timeout -k 10 300 python -u bench.py --config $cfg --erase-pattern download --no-traffic --cpu-seconds 0 --no-host-path > $O/bench_c${cfg}_download.json 2> $O/bench_c${cfg}_download.err || { echo "bench c$cfg failed"; tail -20 $O/bench_c${cfg}_download.err; exit 1; }
  python - $O/bench_c${cfg}_download.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d["roofline"]
print(d["config"]["baseline_config"], d["value"], r["frac"], r["leg_ms"], d["config"]["patterns"]["lost_data_shares_histogram"])
PY
done
