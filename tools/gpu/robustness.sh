#!/bin/bash
# Robustness pass on the current code: the differential fuzz over two seeds
# (every host and device entry point against the oracle), the JIT churn fuzz,
# and the RCCL process-group sequence at one rank.
# usage (via gpurun): bash tools/gpu/robustness.sh OUTDIR [SECONDS] [SEED1] [SEED2]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}; secs=${2:-200}; mkdir -p $out
export TMPDIR=/tmp
for seed in ${3:-7101} ${4:-7202}; do
  timeout -k 10 $((secs + 100)) python tools/fuzz.py --seconds $secs --seed $seed > $out/fuzz_$seed.json 2> $out/fuzz_$seed.err || { tail -5 $out/fuzz_$seed.err; exit 1; }
  tail -1 $out/fuzz_$seed.json
done
timeout -k 10 300 python tools/jit_fuzz.py > $out/jit_fuzz.jsonl 2> $out/jit_fuzz.err || { tail -5 $out/jit_fuzz.err; exit 1; }
tail -2 $out/jit_fuzz.jsonl
timeout -k 10 200 python bench.py --dist-backend nccl --force-pg --steps 20 --warmup 5 --minimal > $out/nccl_force_pg.json 2> $out/nccl.err || exit $?
python3 -c "import json;d=json.loads(open('$out/nccl_force_pg.json').read().strip().splitlines()[-1]);print(d['value'], d['launch']['backend'], d['launch']['pg_ranks'], d['settle'])"
