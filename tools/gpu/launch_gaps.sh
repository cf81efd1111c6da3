#!/bin/bash
# Gaps between consecutive kernels of the default bench's timed steps
# (rocprofv3 kernel trace), and the default line with HIP_FORCE_DEV_KERNARG=1.
# usage: tools/gpu/launch_gaps.sh OUTDIR
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-gaps}; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 40 --warmup 5 --no-host-path --no-traffic --cpu-seconds 0 --minimal > $O/traced_bench.json 2> $O/traced_bench.err || { tail $O/traced_bench.err; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, statistics, json
o = sys.argv[1]
f = glob.glob(o + "/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
k = [r for r in rows if "rs_apply_perm<4, 2" in r["Kernel_Name"]]
gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(k, k[1:])]
gaps = [g / 1000 for g in gaps if g < 100000]  # us, same-stream back-to-back only
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in k]
res = {"kernels": len(k), "gap_us_median": statistics.median(gaps), "gap_us_p10": sorted(gaps)[len(gaps) // 10],
       "gap_us_p90": sorted(gaps)[9 * len(gaps) // 10], "dur_us_median": statistics.median(dur),
       "kernarg_fields": {x: k[0].get(x) for x in ("Kernel_Name", "Private_Segment_Size", "Group_Segment_Size", "Workgroup_Size", "Grid_Size") if x in k[0]}}
print(json.dumps(res))
open(o + "/gaps.json", "w").write(json.dumps(res, indent=1))
PY
find $O/trace -name "*kernel_trace.csv" -delete
for v in 0 1; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python bench.py --no-host-path --no-traffic --cpu-seconds 0 > $O/bench_kernarg$v.json 2> $O/bench_kernarg$v.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/bench_kernarg$v.json').read().strip().splitlines()[-1]); print('HIP_FORCE_DEV_KERNARG=$v', d['value'], d['roofline']['frac'], d['roofline']['leg_ms'])"
done
timeout -k 10 120 tools/_build/gapbench 40 5 > $O/gapbench.txt 2>&1; rc=$?
cat $O/gapbench.txt; exit $rc
