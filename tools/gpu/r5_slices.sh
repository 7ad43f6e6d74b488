#!/bin/bash
# Round-5 host-slice A/B on ONE box: the headline bench in three CPU
# placements, interleaved x${REPS:-3}:
#   node   - the default: the GPU's whole NUMA node (threads float over 128 CPUs under the quota)
#   c16    - --cpus-per-rank -1: the quota-sized slice, 16 lowest CPU ids (16 physical cores)
#   smt32  - --cpus-per-rank 32 --slice-smt: 16 physical cores + their SMT siblings, the share
#            each of 4 ranks owns on a 64-core / 128-thread socket of an 8-GPU node
# Each JSON line carries per-stage cores, context switches per stage and the slice's softirq.
# EXTRA="..." adds bench.py args to every run; SETS="node smt32" picks placements.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/slices
mkdir -p $out
runs=$out/runs${TAG:+_$TAG}.jsonl
: > $runs

{
  echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
  echo "affinity: $(python -c 'import os; print(len(os.sched_getaffinity(0)))')"
  for n in /sys/devices/system/node/node*; do echo "$(basename $n): $(cat $n/cpulist)"; done
  echo "cpu0 siblings: $(cat /sys/devices/system/cpu/cpu0/topology/thread_siblings_list)"
  echo "cpu0 L3 shared: $(cat /sys/devices/system/cpu/cpu0/cache/index3/shared_cpu_list 2>/dev/null)"
  echo "cpu16 L3 shared: $(cat /sys/devices/system/cpu/cpu16/cache/index3/shared_cpu_list 2>/dev/null)"
  grep -m1 "model name" /proc/cpuinfo
} > $out/topology.txt
cat $out/topology.txt

one() {  # label, seconds, bench args...
  local label=$1 secs=$2
  shift 2
  timeout -k 10 $secs python bench.py "$@" $EXTRA > $out/one.jsonl 2> $out/$label.err || {
    echo "FAILED $label"; tail -5 $out/$label.err; return 1; }
  python - "$label" "$runs" <<'PY'
import json, sys
r = json.loads(open('gpurun_out/slices/one.jsonl').read().strip().splitlines()[-1])
r['label'] = sys.argv[1]
open(sys.argv[2], 'a').write(json.dumps(r) + '\n')
print(sys.argv[1], r['value'], 'p50', r.get('p50_latency_ms'), 'p99', r.get('p99_latency_ms'),
      'cores', r['cpu_cores_busy_rank0'], r['cpu_cores_by_stage_rank0'],
      'ctx', r.get('ctx_k_per_s_rank0'), 'slice', r.get('slice_cores_rank0'),
      'cpus', r['cpus_pinned_rank0'], 'spread', r['step_rate_spread']['range_pct'], flush=True)
PY
}

for i in $(seq 1 ${REPS:-3}); do
  for s in ${SETS:-node c16 smt32}; do
    case $s in
      node) one node_$i 240 --steps 20 --warmup 5 || exit 1 ;;
      c16) one c16_$i 240 --steps 20 --warmup 5 --cpus-per-rank -1 || exit 1 ;;
      smt32) one smt32_$i 240 --steps 20 --warmup 5 --cpus-per-rank 32 --slice-smt || exit 1 ;;
      smt16) one smt16_$i 240 --steps 20 --warmup 5 --cpus-per-rank 16 --slice-smt || exit 1 ;;
    esac
  done
done
