#!/bin/bash
# Short vs long timed regions of the default line, the GPU's clocks and power
# cap, and a kernel trace of the driver's exact step count.
# usage (via gpurun): bash tools/gpu/ramp.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}
mkdir -p "$out"
export TMPDIR=/tmp
(amd-smi metric -c -p -g 0 > "$out/amdsmi_metric.txt" 2>&1; \
 amd-smi static -l -g 0 > "$out/amdsmi_static.txt" 2>&1; \
 for f in /sys/class/drm/card*/device/pp_dpm_sclk /sys/class/drm/card*/device/pp_dpm_mclk \
          /sys/class/drm/card*/device/power_dpm_force_performance_level \
          /sys/class/drm/card*/device/hwmon/hwmon*/power1_cap; do
   [ -r "$f" ] && { echo "== $f"; cat "$f"; }; done > "$out/sysfs.txt" 2>&1) || true
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --minimal > "$out/s20_$i.json" 2>> "$out/err.log" || exit $?
done
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 10 --minimal > "$out/s200_$i.json" 2>> "$out/err.log" || exit $?
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof20" -o run -- \
  python3 bench.py --steps 20 --warmup 5 --minimal --no-check > "$out/prof20.json" 2>> "$out/err.log" || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof200" -o run -- \
  python3 bench.py --steps 200 --warmup 10 --minimal --no-check > "$out/prof200.json" 2>> "$out/err.log" || exit $?
python3 - "$out" <<'PY'
import json, sys, glob
out = sys.argv[1]
for f in sorted(glob.glob(out + "/s*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["roofline"]["gpu_ms_per_step"], d["ms_per_step"])
PY
