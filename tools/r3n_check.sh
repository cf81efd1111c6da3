#!/bin/bash
# Checkpoint: the driver's round-end sequence, the download-pattern host
# decode, JIT churn fuzz, single calls.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3n; mkdir -p $O
bash tools/round_check.sh || exit $?
for a in "2 3 262144" "4 6 1048576" "16 24 8388608"; do
  for op in encode decode; do
    for m in pageable pinned; do
      timeout -k 10 60 ./tools/_build/callprobe $a 400 $op $m >> $O/callprobe.jsonl 2>&1 || { echo "callprobe $a $op $m failed"; tail -3 $O/callprobe.jsonl; exit 1; }
    done
  done
done
cat $O/callprobe.jsonl
timeout -k 10 300 python -u bench.py --config 5 --erase-pattern download --no-traffic --cpu-seconds 0 > $O/bench_c5_download_host.json 2> $O/bench_c5_download_host.err || { echo "bench failed"; tail -20 $O/bench_c5_download_host.err; exit 1; }
python - $O/bench_c5_download_host.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["value"], d["roofline"]["frac"], d["roofline"]["leg_ms"], json.dumps(d.get("pcie_inclusive"))[:600])
PY
timeout -k 10 300 python -u bench.py --config 5 --no-traffic --cpu-seconds 0 > $O/bench_c5_fixed_host.json 2> $O/bench_c5_fixed_host.err || { echo "bench failed"; tail -20 $O/bench_c5_fixed_host.err; exit 1; }
python - $O/bench_c5_fixed_host.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["value"], d["roofline"]["frac"], json.dumps(d.get("pcie_inclusive"))[:400])
PY
STORB_RS_JIT_MAX=32 timeout -k 10 400 python -u tools/jit_fuzz.py 10000 2000 > $O/jit_fuzz.jsonl 2>&1 || { echo "fuzz failed"; tail -5 $O/jit_fuzz.jsonl; exit 1; }
tail -1 $O/jit_fuzz.jsonl
