set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6y
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/valu64_probe.hip -o /tmp/valu64 2>/dev/null || exit 1
timeout -k 10 90 /tmp/valu64 > gpurun_out/r6y/valu64.txt 2>&1 || exit $?
cat gpurun_out/r6y/valu64.txt
for z in 1 0; do
  STORB_RS_ZC_BATCH=$z timeout -k 10 120 python tools/hostpath.py > gpurun_out/r6y/hostpath_zc$z.json 2> gpurun_out/r6y/hostpath_zc$z.err || exit $?
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1], {k:v for k,v in d.items() if 'value' in k})" gpurun_out/r6y/hostpath_zc$z.json
done
