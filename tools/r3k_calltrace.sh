#!/bin/bash
# (1) host-registration probe (no device work on freed memory); (2) stage
# timeline of the single calls; (3) mixed-row descriptor decode; (4) the
# download-pattern bench legs.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3k; mkdir -p $O
timeout -k 10 120 python -u tools/register_probe.py > $O/register_probe.json 2>&1 || { echo "probe failed"; tail -20 $O/register_probe.json; exit 1; }
python - $O/register_probe.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read()[open(sys.argv[1]).read().index('{'):])
print("unregister_rc", d["unregister_rc"], "after", [(a["hipHostGetDevicePointer"], a["memoryType"]) for a in d["after_unregister"]][:3])
for f in d["fresh_arrays"]: print(f)
PY
for a in "4 6 1048576" "2 3 262144" "16 24 8388608"; do
  for op in encode decode; do
    echo "== $a $op pageable" >> $O/calltrace.txt
    timeout -k 10 60 ./tools/_build/callprobe_trace $a 300 $op pageable >> $O/calltrace.txt 2>&1 || { echo "callprobe_trace failed"; tail -5 $O/calltrace.txt; exit 1; }
  done
done
cat $O/calltrace.txt
timeout -k 10 120 ./tools/_build/descbench 20 > $O/descbench.txt 2>&1 || { echo "descbench failed"; tail $O/descbench.txt; exit 1; }
head -1 $O/descbench.txt; grep -E "mixed-row launch, cap 0|host time|uniform" $O/descbench.txt
for cfg in "5" "6" "2"; do
  timeout -k 10 300 python -u bench.py --config $cfg --erase-pattern download --no-traffic --cpu-seconds 0 --no-host-path > $O/bench_c${cfg}_download.json 2> $O/bench_c${cfg}_download.err || { echo "bench c$cfg failed"; tail -20 $O/bench_c${cfg}_download.err; exit 1; }
  python - $O/bench_c${cfg}_download.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d["roofline"]
print(d["config"]["baseline_config"], d["value"], r["frac"], r["leg_ms"], d["config"]["patterns"]["lost_data_shares_histogram"])
PY
done
