#!/bin/bash
# Final code: the test order that faulted twice this round (patterns ->
# async -> jit -> parity in one process; the registration checks now run in
# child processes), then a longer differential fuzz.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_patterns.py tests/test_gpu_async.py tests/test_gpu_jit.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/fuzz.py --seconds 120 --seed 61 > $O/fuzz.json 2>&1 || { echo "fuzz failed"; tail -20 $O/fuzz.json; exit 1; }
tail -1 $O/fuzz.json
