#!/bin/bash
# GPU-box: GPU tests, then the default bench and a sweep of host-path knobs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
SWEEP=${SWEEP:-"--replicas-per-gpu 2|--replicas-per-gpu 4|--replicas-per-gpu 2 --batch 512|--replicas-per-gpu 4 --batch 512 --decode-threads 4"}
IFS='|'
for args in $SWEEP; do
  unset IFS
  timeout -k 10 300 python bench.py --steps 200 $args > gpurun_out/bench_sweep.log 2>&1 || exit $?
  echo "$args: $(tail -1 gpurun_out/bench_sweep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"], d["device_ms_p50"], d["batch_images_mean"], d["json_mb_per_s_rank0"], d["rank0_thread_s"])')"
  IFS='|'
done
