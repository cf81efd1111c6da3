#!/bin/bash
# A/B: k < 8 table kernels reading their tables as scalar loads (new) vs
# per-lane vector loads (old), on the headline config 2 (RS(4,2)), interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3q; mkdir -p $O
for i in 1 2 3 4; do
  for v in old new; do
    timeout -k 10 120 python -u tools/lib_ab.py tools/_build/ab/$v/libstorb_rs.so --no-host-path --no-traffic --cpu-seconds 0 --steps 400 > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { echo "bench $v failed"; tail -5 $O/bench_${v}_$i.err; exit 1; }
    python - $O/bench_${v}_$i.json $v <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d["roofline"]
print(sys.argv[2], d["value"], r["frac"], r["leg_ms"])
PY
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
