#!/bin/bash
# What the driver runs at round end, on a GPU box: the -m gpu suite, smoke(),
# and the default bench line (with its wall time). Outputs in gpurun_out/.
# usage (via gpurun): bash tools/round_check.sh
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/rc_gputest.log 2>&1
rc=$?
tail -2 gpurun_out/rc_gputest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/rc_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/rc_smoke.log
t0=$(date +%s.%N)
timeout -k 10 300 python bench.py > gpurun_out/rc_bench.json 2> gpurun_out/rc_bench.err || exit $?
t1=$(date +%s.%N)
python - "$t0" "$t1" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/rc_bench.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("bench wall %.1f s" % (float(sys.argv[2]) - float(sys.argv[1])), d["value"], d["unit"],
      "frac", r["frac"], "traffic", r["traffic"], "cpu", (d.get("cpu_baseline") or {}).get("value"),
      "decode_pinned", (d.get("pcie_inclusive") or {}).get("decode_pinned_value"))
dl = d.get("download_decode") or {}
print("download", dl.get("value"), (dl.get("roofline") or {}).get("frac"),
      (dl.get("roofline") or {}).get("traffic_vs_algorithmic"))
cb = d.get("cpu_baseline") or {}
print("cpu", cb.get("value"), (cb.get("arithmetic_only") or {}).get("value"), cb.get("thread"))
for g in (d.get("shim_path") or {}).get("geometries", []):
    print("shim", g["k"], g["m_total"], {x: g[x]["median_us"] for x in ("encode_call", "encode_shim", "decode_call", "decode_shim")})
PY
