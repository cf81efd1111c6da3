#!/bin/bash
# Kernel variants + product descriptor path + parity tests + the default bench line.
# usage: tools/gpu/check.sh OUTDIR [pytest files...]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-check}; shift; mkdir -p $O
TESTS=${*:-tests/test_gpu_patterns.py tests/test_gpu_parity.py}
timeout -k 10 180 tools/_build/mixbench 25 16 > $O/mixbench16.txt 2>&1 &&
timeout -k 10 180 tools/_build/mixbench 25 32 > $O/mixbench32.txt 2>&1 &&
timeout -k 10 120 tools/_build/descbench 20 32 > $O/descbench32.txt 2>&1 &&
timeout -k 10 120 tools/_build/descbench 20 16 > $O/descbench16.txt 2>&1 || { echo "bench tools failed"; exit 1; }
grep -E "product|G16|same shape|uniform" $O/mixbench16.txt $O/mixbench32.txt $O/descbench32.txt $O/descbench16.txt
timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "frac", r["frac"], "traffic", r["traffic"])
print("cpu", json.dumps(d.get("cpu_baseline"))[:900])
print("download", json.dumps(d.get("download_decode"))[:900])
p = d.get("pcie_inclusive") or {}
print("pcie", {k: p.get(k) for k in ("value", "pinned_value", "decode_value", "decode_pinned_value", "decode_download_value", "decode_pinned_download_value")})
for g in (d.get("shim_path") or {}).get("geometries", []):
    print("shim", g["k"], g["m_total"], {x: g[x]["median_us"] for x in ("encode_call", "encode_shim", "decode_call", "decode_shim")})
PY
