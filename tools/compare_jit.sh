#!/bin/bash
# A/B of the run-time-compiled bit-sliced decode against the table kernel on
# decodes the policy leaves to the table kernel (config 3's RS(8,4) with 3
# lost; RS(16,8) with 2 lost): STORB_RS_JIT=0 vs =always. Bench lines in
# gpurun_out/cmp_<cfg>_<mode>.log.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in 0 always; do
  STORB_RS_JIT=$v timeout -k 10 200 python3 bench.py --config 3 --cpu-seconds 0 --no-host-path \
    --no-traffic > gpurun_out/cmp_c3_$v.log 2>&1
  STORB_RS_JIT=$v timeout -k 10 200 python3 bench.py --config 5 --erase 2 --cpu-seconds 0 \
    --no-host-path --no-traffic > gpurun_out/cmp_c5e2_$v.log 2>&1
done
echo done
