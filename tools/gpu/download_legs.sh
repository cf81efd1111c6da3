#!/bin/bash
# Config 5 / 6 with download patterns: the bench line with live FETCH/WRITE
# traffic of the descriptor decode leg, and a rocprof --stats trace of each.
# usage: tools/gpu/download_legs.sh OUTDIR
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-dl}; mkdir -p $O
for c in 5 6; do
  timeout -k 10 400 python bench.py --config $c --erase-pattern download --no-host-path --cpu-seconds 0 > $O/bench_c${c}_download.json 2> $O/bench_c${c}_download.err || { tail $O/bench_c${c}_download.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_c${c}_download.json').read().strip().splitlines()[-1]); r=d['roofline']; print('config $c', d['value'], r['frac'], r['leg_ms'], json.dumps(r.get('traffic_by_leg')))"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c${c} -o run -- python3 bench.py --config $c --erase-pattern download --no-host-path --no-traffic --cpu-seconds 0 > $O/traced_c${c}.json 2>&1 || exit 1
  find $O/trace_c${c} -name "*kernel_trace.csv" -delete
  grep -h "desc_mix" $(find $O/trace_c${c} -name "*kernel_stats.csv") | cut -c1-160
done
