#!/bin/bash
# The default bench line's shim_path, with the (4, 6) calls repeated with the
# calling thread on the GPU's NUMA node and on the other node; 2 runs.
# usage: tools/gpu/shim_numa.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-numa}; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-traffic --cpu-seconds 2 > $O/bench$i.json 2> $O/bench$i.err || { tail $O/bench$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench$i.json').read().strip().splitlines()[-1])
for g in d['shim_path']['geometries']:
    print(g['k'], g['m_total'], {x: g[x]['median_us'] for x in ('encode_call','encode_shim','decode_call','decode_shim')})
    if 'numa' in g: print(json.dumps(g['numa']))
print('pinned decode', d.get('pcie_inclusive',{}).get('decode_pinned_value'), 'value', d['value'])"
done
