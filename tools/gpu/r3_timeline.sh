#!/bin/bash
# GPU box: two default bench.py runs with the 100 ms diagnostic timeline (lines a throughput sag up
# with per-stage cores, cgroup throttling, queue depth and broker output)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 240 python bench.py --timeline gpurun_out/tl$i.jsonl --timeline-ms 100 "$@" \
    > gpurun_out/tl$i.log 2>&1 || { tail -20 gpurun_out/tl$i.log; exit 1; }
  grep '^{' gpurun_out/tl$i.log | tail -1
done
