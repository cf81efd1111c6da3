set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --force-pg --dist-backend nccl --steps 50 --warmup 5 --no-traffic --cpu-seconds 3 --no-host-path > gpurun_out/r3a_nccl_force.json 2> gpurun_out/r3a_nccl_force.err || { echo "nccl force failed $?"; tail -20 gpurun_out/r3a_nccl_force.err; exit 1; }
tail -c 600 gpurun_out/r3a_nccl_force.json
timeout -k 10 400 python -u bench.py > gpurun_out/r3a_bench.json 2> gpurun_out/r3a_bench.err || { echo "bench failed $?"; tail -20 gpurun_out/r3a_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r3a_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['frac']);print(json.dumps(d.get('shim_path'))[:3000])"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a_gputest.log 2>&1
rc=$?; tail -3 gpurun_out/r3a_gputest.log; exit $rc
