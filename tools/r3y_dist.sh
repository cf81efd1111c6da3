#!/bin/bash
# Multi-rank launch paths on the final code: the RCCL process-group sequence
# forced at one rank, and a 2-rank gloo rehearsal sharing the one GPU.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3y; mkdir -p $O
timeout -k 10 200 python -u bench.py --dist-backend nccl --force-pg --steps 50 --warmup 5 > $O/nccl_force_world1.json 2> $O/nccl.err || { echo "nccl failed"; tail -20 $O/nccl.err; exit 1; }
tail -1 $O/nccl_force_world1.json | cut -c1-200
STORB_BENCH_DEVICE=0 timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 50 --warmup 5 > $O/gloo_spawn2.json 2> $O/gloo.err || { echo "gloo failed"; tail -20 $O/gloo.err; exit 1; }
tail -1 $O/gloo_spawn2.json | cut -c1-200
