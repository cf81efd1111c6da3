#!/bin/bash
# Round 3: per-chunk erasure patterns (download), GPU suite, rocprof of the
# download decode. usage (via gpurun): bash tools/r3b_check.sh
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3b
O=gpurun_out/r3b
timeout -k 10 300 python -u -m pytest tests/test_gpu_patterns.py tests/test_rust_binding.py -x -q --timeout 120 --timeout-method thread > $O/patterns_tests.log 2>&1 || { tail -30 $O/patterns_tests.log; exit 1; }
tail -1 $O/patterns_tests.log
for cfg in "5" "6" "2"; do
  timeout -k 10 300 python -u bench.py --config $cfg --erase-pattern download --no-traffic --cpu-seconds 3 > $O/bench_c${cfg}_download.json 2> $O/bench_c${cfg}_download.err || { echo "bench c$cfg failed"; tail -20 $O/bench_c${cfg}_download.err; exit 1; }
  python - $O/bench_c${cfg}_download.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d["roofline"]; p=d.get("pcie_inclusive") or {}
print(d["config"]["baseline_config"], d["value"], r["frac"], r["leg_ms"], d["config"]["patterns"], r["jit"],
      {x: p.get(x) for x in ("decode_value","decode_pinned_value","decode_download_value","decode_pinned_download_value")})
PY
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5_download -o run -- python3 bench.py --config 5 --erase-pattern download --no-host-path --no-traffic --cpu-seconds 0 > $O/trace_c5_download.log 2>&1 || { echo "trace failed"; tail -20 $O/trace_c5_download.log; exit 1; }
echo traced
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; tail -3 $O/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
python -c "import json;d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]);print('default',d['value'],d['roofline']['frac'],d['roofline']['traffic'])"
