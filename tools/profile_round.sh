#!/bin/bash
# Collects the round profiles on a GPU box into gpurun_out/prof_<ROUND>/:
#   trace/  rocprofv3 --kernel-trace --stats of `python3 bench.py --no-host-path`
#   fetch/, write/  separate FETCH_SIZE and WRITE_SIZE passes (TCC slots, MI355X_MICROARCH.md)
#   bench_*.log  the bench lines (traced and untraced)
# Then, back in the container:
#   python3 profiles/summarize.py <ROUND> gpurun_out/prof_<ROUND>/{trace,fetch,write} --kernel ...
# usage (via gpurun): bash tools/profile_round.sh r1
set -euo pipefail
ROUND=${1:-r1}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/prof_$ROUND
rm -rf "$OUT" && mkdir -p "$OUT"
KSUB="rs_apply_perm<4, 2, 256, 1, false, 4, false, false, false>"
# --no-host-path: the PCIe legs launch the same kernel on host-staged batches
# (18 us .. 3.6 ms each), which would blend into its average; this run's own
# bench line (bench_traced.log) is the one the stats are compared with.
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 bench.py --no-host-path > "$OUT/bench_traced.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" \
  -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-host-path \
  > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" \
  -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-host-path \
  > "$OUT/write.log" 2>&1
echo "$KSUB" > "$OUT/kernel.txt"
timeout -k 10 300 python3 bench.py > "$OUT/bench_untraced.log" 2>&1
echo done
