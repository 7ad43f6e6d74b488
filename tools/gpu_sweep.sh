#!/bin/bash
# GPU-box: bench.py over a '|'-separated list of argument sets (SWEEP), one summary line each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SWEEP=${SWEEP:-"--replicas-per-gpu 4"}
IFS='|'
i=0
for args in $SWEEP; do
  unset IFS
  i=$((i+1))
  timeout -k 10 300 python bench.py ${COMMON:-} $args > gpurun_out/sweep_$i.log 2>&1 || { echo "FAILED: $args"; tail -5 gpurun_out/sweep_$i.log; exit 1; }
  echo "$args: $(tail -1 gpurun_out/sweep_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "p50", d["p50_latency_ms"], "dev", d["device_ms_p50"], "bimg", d["batch_images_mean"], "MBs", d["json_mb_per_s_rank0"], "cpu", d.get("cpu_cores_busy_rank0"), d["rank0_thread_s"])')"
  IFS='|'
done
