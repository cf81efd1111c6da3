#!/bin/bash
# Environment A/B of bench.py workloads: every (case, env spec) pair run
# REPS times, interleaved (rounds outer), one bench line each in
# gpurun_out/env_<case>_<spec>_<round>.log. An env spec is a
# '+'-separated list of VAR=VALUE ("base" = no extra variables).
# usage: bash tools/env_ab.sh "c2 c3" "base STORB_RS_TABLE_T=64+STORB_RS_WG_PER_CU=20" 2
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
CASES=${1:-"c2"}
SPECS=${2:-"base"}
REPS=${3:-2}
for ((r = 0; r < REPS; r++)); do
  for c in $CASES; do
    case $c in
      c2) args="" ;;
      c3) args="--config 3" ;;
      c4) args="--config 4" ;;
      c5) args="--config 5" ;;
      c5e*) args="--config 5 --erase ${c#c5e}" ;;
      c6e*) args="--config 6 --erase ${c#c6e}" ;;
      c7) args="--config 7" ;;
      c7e*) args="--config 7 --erase ${c#c7e}" ;;
    esac
    for sp in $SPECS; do
      envs=()
      [ "$sp" != base ] && IFS='+' read -r -a envs <<< "$sp"
      tag=${sp//[=+,]/_}
      env "${envs[@]}" timeout -k 10 200 python3 bench.py $args --cpu-seconds 0 --no-host-path \
        --no-traffic > "gpurun_out/env_${c}_${tag}_$r.log" 2>&1
      echo "$r $c $sp done"
    done
  done
done
