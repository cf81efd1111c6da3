#!/bin/bash
# Mixed-row descriptor launch + spin waits in the single-chunk calls.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3j; mkdir -p $O
timeout -k 10 120 ./tools/_build/descbench 20 > $O/descbench.txt 2>&1 || { echo "descbench failed"; tail $O/descbench.txt; exit 1; }
cat $O/descbench.txt
for a in "2 3 262144" "4 6 1048576" "16 24 8388608"; do
  for op in encode decode; do
    for m in pageable pinned; do
      timeout -k 10 60 ./tools/_build/callprobe $a 400 $op $m >> $O/callprobe.jsonl 2>&1 || { echo "callprobe $a $op $m failed"; tail -3 $O/callprobe.jsonl; exit 1; }
    done
  done
done
cat $O/callprobe.jsonl
timeout -k 10 500 python -u -m pytest tests/test_gpu_patterns.py tests/test_gpu_async.py tests/test_gpu_jit.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in "5" "6"; do
  timeout -k 10 300 python -u bench.py --config $cfg --erase-pattern download --no-traffic --cpu-seconds 0 --no-host-path > $O/bench_c${cfg}_download.json 2> $O/bench_c${cfg}_download.err || { echo "bench c$cfg failed"; tail -20 $O/bench_c${cfg}_download.err; exit 1; }
  python - $O/bench_c${cfg}_download.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d["roofline"]
print(d["config"]["baseline_config"], d["value"], r["frac"], r["leg_ms"], d["config"]["patterns"]["lost_data_shares_histogram"])
PY
done
