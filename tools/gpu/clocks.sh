#!/bin/bash
# amd-smi / sysfs clock and power readings of the visible GPU, and the
# effective gfx clock per launch (GRBM_GUI_ACTIVE / 8 XCDs / duration) over a
# short default run.  usage (via gpurun): bash tools/gpu/clocks.sh OUTDIR
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=${1:?outdir}
mkdir -p "$out"
export TMPDIR=/tmp
(timeout 30 amd-smi list --json > "$out/amdsmi_list.json" 2>&1
 timeout 30 amd-smi metric -c -p --json > "$out/amdsmi_metric.json" 2>&1
 timeout 30 amd-smi static -l --json > "$out/amdsmi_static_limit.json" 2>&1
 python3 -c "import torch;print(torch.cuda.get_device_properties(0).pci_bus_id if hasattr(torch.cuda.get_device_properties(0),'pci_bus_id') else None)" > "$out/busid.txt" 2>&1
 ls -la /sys/bus/pci/devices/ > "$out/pci_ls.txt" 2>&1) || true
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$out/grbm" -o run -- \
  python3 bench.py --steps 20 --warmup 5 --minimal --no-check > "$out/grbm.json" 2>> "$out/err.log" || exit $?
