#!/bin/bash
# Config 3's <8,3> decode on one-wave workgroups (rs_device.hpp PermShape):
# the -m gpu suite, then a kernel trace of bench.py --config 3 and the
# default line. Outputs in gpurun_out/r6s_c3/.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r6s_c3
rm -rf "$OUT" && mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/gputest.log" 2>&1 || { tail -30 "$OUT/gputest.log"; exit 1; }
tail -2 "$OUT/gputest.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_config3" \
  -o run -- python3 bench.py --no-host-path --no-traffic --cpu-seconds 0 --config 3 \
  > "$OUT/bench_config3.log" 2>&1 || exit 2
find "$OUT/trace_config3" -name "*kernel_trace.csv" -delete
grep -h "rs_apply_perm" $(find "$OUT/trace_config3" -name "*kernel_stats.csv") | cut -c1-200
timeout -k 10 300 python3 bench.py --config 3 --cpu-seconds 0 > "$OUT/bench_config3_plain.log" 2>&1 || exit 3
tail -c 400 "$OUT/bench_config3_plain.log"
