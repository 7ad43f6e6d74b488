#!/bin/bash
# GPU-box: end-to-end bench (bench.py) + short GPU test pass. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --batch 1024 --source-parallelism 4 > gpurun_out/bench_b1024.log 2>&1
rc=$?; echo "bench1024 rc=$rc"; tail -3 gpurun_out/bench_b1024.log
exit $rc
