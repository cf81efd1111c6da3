#!/bin/bash
# Descriptor / table-kernel launch-shape sweeps (tools/mixbench.hip,
# tools/k32_tune.hip) and the product descriptor path (tools/descbench.cpp),
# then the pattern tests that pin the kernels bit-exact to the oracle.
# usage: tools/gpu/kernel_sweeps.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
# tools/_build does not travel to the box (.gpurunignore): build there
make -s -j4 -C tools mixbench k32_tune descbench > /dev/null || exit 1
O=gpurun_out/${1:-sweeps}; mkdir -p $O
timeout -k 10 120 tools/_build/mixbench 25 16 > $O/mixbench16.txt 2>&1 && cat $O/mixbench16.txt &&
timeout -k 10 120 tools/_build/mixbench 25 32 > $O/mixbench32.txt 2>&1 && cat $O/mixbench32.txt &&
timeout -k 10 240 tools/_build/k32_tune 15 > $O/k32_tune.txt 2>&1 && cat $O/k32_tune.txt &&
timeout -k 10 120 tools/_build/descbench 20 32 > $O/descbench32.txt 2>&1 && cat $O/descbench32.txt &&
timeout -k 10 120 tools/_build/descbench 20 16 > $O/descbench16.txt 2>&1 && cat $O/descbench16.txt &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_lifetime.py tests/test_gpu_runtime.py tests/test_gpu_patterns.py tests/test_gpu_async.py tests/test_gpu_jit.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; exit $rc
