#!/bin/bash
# Collects a round's profiles on a GPU box into gpurun_out/prof_<ROUND>/:
#   trace_<cfg>/   rocprofv3 --kernel-trace --stats of bench.py for each leg set
#                  below (--no-host-path: the PCIe legs launch the same kernels
#                  on host-staged batches and would blend into the averages)
#   bench_<cfg>.log  the bench line of that traced run
#   bench_default.log  the untraced default bench (the driver's command; its
#                  roofline.traffic comes from its own live FETCH/WRITE passes)
# Then, back in the container: python3 profiles/summarize.py <ROUND> gpurun_out/prof_<ROUND>
# usage (via gpurun): bash tools/profile_round.sh r2
set -euo pipefail
ROUND=${1:-r2}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/prof_$ROUND
rm -rf "$OUT" && mkdir -p "$OUT"
trace() {  # name, bench args...
  local name=$1
  shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$name" \
    -o run -- python3 bench.py --no-host-path --no-traffic --cpu-seconds 0 "$@" \
    > "$OUT/bench_$name.log" 2>&1
  # keep the --stats summary (what profiles/summarize.py reads); the full
  # per-dispatch trace would push gpurun_out past its copy-back limit
  find "$OUT/trace_$name" -name "*kernel_trace.csv" -delete
  echo "traced $name"
}
trace config2
trace config5 --config 5
trace config5_erase8 --config 5 --erase 8
trace config6_erase16 --config 6 --erase 16
trace config3 --config 3
trace config4 --config 4
trace config7 --config 7
trace config7_erase32 --config 7 --erase 32
trace config2_download --erase-pattern download
trace config5_download --config 5 --erase-pattern download
trace config6_download --config 6 --erase-pattern download
timeout -k 10 400 python3 bench.py > "$OUT/bench_default.log" 2>&1
echo "default bench done"
echo done
