#!/bin/bash
# 64-bit shifts in the bit-slice transposition (rs_bitslice_core.h
# STORB_BS_SHIFT64): issue-rate probe, then the bit-sliced GPU tests on the
# library built with it, then bstune A/B (0 / 1 builds, interleaved runs).
# usage (via gpurun): bash tools/gpu/shift64_ab.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}
mkdir -p $out
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/valu64_probe.hip -o /tmp/valu64 2>/dev/null || exit 1
timeout -k 10 60 /tmp/valu64 > $out/valu64.txt 2>&1 || exit $?
cat $out/valu64.txt
for v in 0 1; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -Istorb_amd/csrc -DSTORB_BS_SHIFT64=$v tools/bstune.hip \
    -o /tmp/bst$v 2>/dev/null &
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_jit.py -m gpu -x -q \
  -k "bitslice or jit" --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
wait
for r in 1 2; do
  for v in 0 1; do
    BSTUNE_KSPLIT=1 timeout -k 10 120 /tmp/bst$v 5 1 > $out/enc_s${v}_$r.txt 2>&1 || exit $?
    echo "== SHIFT64=$v round $r"; cat $out/enc_s${v}_$r.txt
  done
done
for v in 0 1; do
  BSTUNE_KSPLIT=1 timeout -k 10 120 /tmp/bst$v 5 5 > $out/dec_s${v}.txt 2>&1 || exit $?
  echo "== decodes SHIFT64=$v"; cat $out/dec_s${v}.txt
done
