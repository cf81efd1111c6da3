#!/bin/bash
# Encode + piece ids in one kernel (rs_encode_hash.hip): its GPU tests, then
# the default bench line's shard_hashing object (fused vs two kernels).
# usage: tools/gpu/fused_hash.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-fh}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_blake3.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python bench.py --no-host-path --no-traffic --cpu-seconds 0 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['frac']); print(json.dumps(d.get('shard_hashing'), indent=1))"
