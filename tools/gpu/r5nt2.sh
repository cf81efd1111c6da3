#!/bin/bash
# Host-path GPU tests on the build with non-temporal batch copies, then the
# batch host paths against the staging-only NT build.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5nt2; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_blake3.py tests/test_gpu_patterns.py \
  tests/test_gpu_runtime.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 \
  || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
bash tools/gpu/hostpath_ab.sh $out 3 storb_amd/lib/ab_nt/libstorb_rs.so storb_amd/lib/libstorb_rs.so
