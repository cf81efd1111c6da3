#!/bin/bash
# Pool accounting (table cache freed with hipFreeAsync vs the old hipFree),
# single-call copy split A/B, then the test order that faulted twice.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3m; mkdir -p $O
timeout -k 10 120 python -u tools/pool_probe.py > $O/pool_probe_new.json 2>&1 || { echo "pool probe failed"; tail -20 $O/pool_probe_new.json; exit 1; }
timeout -k 10 120 python -u tools/pool_probe.py tools/_build/oldpool/libstorb_rs.so > $O/pool_probe_old.json 2>&1 || { echo "pool probe (old) failed"; tail -20 $O/pool_probe_old.json; exit 1; }
cat $O/pool_probe_new.json $O/pool_probe_old.json | grep -v amdgpu.ids
for v in flags p1 p4 p8; do
  for op in encode decode; do
    echo "== $v 4 6 1048576 $op pageable" >> $O/calltrace.txt
    LD_LIBRARY_PATH=tools/_build/$v timeout -k 10 60 ./tools/_build/callprobe_trace 4 6 1048576 300 $op pageable >> $O/calltrace.txt 2>&1 || { echo "callprobe_trace failed"; tail -5 $O/calltrace.txt; exit 1; }
  done
done
grep -E "^==|median_us" $O/calltrace.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_patterns.py tests/test_gpu_async.py tests/test_gpu_jit.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
