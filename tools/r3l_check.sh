#!/bin/bash
# Stream-written slice flags (single calls) and kernel-copied descriptors.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3l; mkdir -p $O
timeout -k 10 120 python -u tools/register_probe.py > $O/register_probe.json 2>&1 || { echo "probe failed"; tail -20 $O/register_probe.json; exit 1; }
python - $O/register_probe.json <<'PY'
import json,sys
t=open(sys.argv[1]).read(); d=json.loads(t[t.index('{'):])
print("registered dev va", d["registered_dev_va"][:3], "torch va", d["torch_tensor_va"][:4])
print("torch after unregister", d["torch_tensors_after_unregister"])
print("new", d["torch_new_tensors"])
PY
for v in flags events; do
  LP=""; [ $v = events ] && LP="tools/_build/evt"
  for a in "4 6 1048576" "2 3 262144"; do
    for op in encode decode; do
      echo "== $v $a $op pageable" >> $O/calltrace.txt
      LD_LIBRARY_PATH=$LP timeout -k 10 60 ./tools/_build/callprobe_trace $a 300 $op pageable >> $O/calltrace.txt 2>&1 || { echo "callprobe_trace failed"; tail -5 $O/calltrace.txt; exit 1; }
    done
  done
done
grep -E "^==|median_us" $O/calltrace.txt
for a in "2 3 262144" "4 6 1048576" "16 24 8388608"; do
  for op in encode decode; do
    for m in pageable pinned; do
      timeout -k 10 60 ./tools/_build/callprobe $a 400 $op $m >> $O/callprobe.jsonl 2>&1 || { echo "callprobe $a $op $m failed"; tail -3 $O/callprobe.jsonl; exit 1; }
    done
  done
done
cat $O/callprobe.jsonl
timeout -k 10 120 ./tools/_build/descbench 20 > $O/descbench.txt 2>&1 || { echo "descbench failed"; tail $O/descbench.txt; exit 1; }
head -1 $O/descbench.txt; grep -E "mixed-row launch, cap 0|host time|uniform" $O/descbench.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_patterns.py tests/test_gpu_async.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --config 5 --erase-pattern download --no-traffic --cpu-seconds 0 --no-host-path > $O/bench_c5_download.json 2> $O/bench_c5_download.err || { echo "bench failed"; tail -20 $O/bench_c5_download.err; exit 1; }
python - $O/bench_c5_download.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d["roofline"]
print(d["config"]["baseline_config"], d["value"], r["frac"], r["leg_ms"])
PY
