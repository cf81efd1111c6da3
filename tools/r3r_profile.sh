#!/bin/bash
# Round 3 profiles: rocprofv3 kernel traces of every bench config (incl. the
# download-pattern ones), the untraced default line, and the JIT fuzz with
# timestamps.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/profile_round.sh r3 > gpurun_out/r3r_profile.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/r3r_profile.log; exit 1; }
tail -3 gpurun_out/r3r_profile.log
mkdir -p gpurun_out/r3r
STORB_RS_JIT_MAX=32 timeout -k 10 300 python -u tools/jit_fuzz.py 10000 2000 > gpurun_out/r3r/jit_fuzz.jsonl 2>&1 || { echo "fuzz failed"; tail -5 gpurun_out/r3r/jit_fuzz.jsonl; exit 1; }
cut -c1-160 gpurun_out/r3r/jit_fuzz.jsonl
