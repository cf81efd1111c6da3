#!/bin/bash
# Shim single calls with the caller on each NUMA node, for staging buffers
# placed by the runtime (default) and pinned to node 0 / node 1
# (STORB_RS_STAGING_NODE).
# usage: tools/gpu/staging_numa.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-snuma}; mkdir -p $O
for st in default 0 1; do
  if [ $st = default ]; then unset STORB_RS_STAGING_NODE; else export STORB_RS_STAGING_NODE=$st; fi
  timeout -k 10 300 python bench.py --no-traffic --no-host-path --cpu-seconds 0 > $O/bench_$st.json 2> $O/bench_$st.err || { tail $O/bench_$st.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$st.json').read().strip().splitlines()[-1])
for g in d['shim_path']['geometries']:
    if 'numa' in g:
        n=g['numa']; print('staging $st', 'gpu node', n['gpu_numa_node'], 'default', g['encode_call']['median_us'], g['decode_call']['median_us'], 'caller on gpu node', n['caller_on_gpu_node'], 'other', n['caller_on_other_node'])"
done
