#!/bin/bash
# Host topology of the GPU box and the single-call latency with the calling
# thread (and the library's copy workers, which inherit its affinity) placed
# on each NUMA node in turn: is the staging copy slow because it crosses
# sockets? (DESIGN.md §5 single calls.)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/numa; mkdir -p $O
{
  echo "nodes online: $(cat /sys/devices/system/node/online)"
  for n in /sys/devices/system/node/node*; do echo "$(basename $n): cpus $(cat $n/cpulist)"; done
  grep -E "Cpus_allowed_list|Mems_allowed_list" /proc/self/status
  for d in /sys/class/drm/card*/device; do
    [ -f $d/numa_node ] && echo "$(basename $(dirname $d)) $(cat $d/uevent | grep PCI_SLOT_NAME) numa_node $(cat $d/numa_node)"
  done
  cat /sys/fs/cgroup/cpu.max 2>/dev/null
  lscpu | grep -E "Model name|Socket|NUMA|^CPU\(s\)"
} > $O/topology.txt 2>&1
cat $O/topology.txt
for n in /sys/devices/system/node/node*; do
  cpus=$(cat $n/cpulist)
  first=${cpus%%,*}
  for op in encode decode; do
    echo "== $(basename $n) ($first...) $op" >> $O/callprobe_numa.txt
    timeout -k 10 60 taskset -c "$cpus" ./tools/_build/callprobe 4 6 1048576 300 $op pageable >> $O/callprobe_numa.txt 2>&1 || { echo "callprobe failed"; tail -3 $O/callprobe_numa.txt; exit 1; }
    timeout -k 10 60 taskset -c "$cpus" ./tools/_build/callprobe 4 6 1048576 300 $op pinned >> $O/callprobe_numa.txt 2>&1 || exit 1
  done
done
cat $O/callprobe_numa.txt
