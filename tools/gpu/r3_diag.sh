#!/bin/bash
# Round-3 diagnosis of the bench throughput slide: host/cgroup facts, then default bench runs
# with a 100 ms timeline (completions, per-stage cores, cgroup throttling, RSS, queue, lag).
set -o pipefail
mkdir -p gpurun_out/diag
{
  echo "== nproc $(nproc)"; cat /sys/fs/cgroup/cpu.max 2>&1; cat /sys/fs/cgroup/cpuset.cpus.effective 2>&1
  cat /sys/fs/cgroup/memory.max 2>&1; cat /sys/fs/cgroup/cpu.stat 2>&1
  python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
  lscpu | head -30; numactl -H 2>&1 | head -20; cat /proc/pressure/cpu 2>&1; cat /proc/pressure/memory 2>&1
  cat /sys/kernel/mm/transparent_hugepage/enabled; cat /proc/sys/kernel/numa_balancing
  uptime
} > gpurun_out/diag/host.txt 2>&1
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --timeline gpurun_out/diag/tl$i.jsonl \
    > gpurun_out/diag/b$i.json 2> gpurun_out/diag/b$i.err || exit $?
  cat /proc/pressure/cpu >> gpurun_out/diag/host.txt
done
