#!/bin/bash
# GPU-box: host topology the host pipeline runs on (CPU share, NUMA nodes, the GPU's node).
set -u
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"
echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
echo "cpuset: $(cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null)"
for n in /sys/devices/system/node/node*; do echo "$n cpus $(cat $n/cpulist)"; done
for d in /sys/class/drm/card*/device; do
  echo "$d numa_node=$(cat $d/numa_node 2>/dev/null) $(grep PCI_SLOT_NAME $d/uevent 2>/dev/null)"
done
grep -m1 "model name" /proc/cpuinfo
head -2 /proc/meminfo
