#!/bin/bash
# GPU-box check script: tests -> forward bench -> rocprofv3 kernel stats. Stops at the first
# GPU fault / abort / timeout (exit codes other than 0/1 from pytest).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python tools/bench_forward.py --model resnet20 > gpurun_out/fwd_r20.log 2>&1 || exit $?
cat gpurun_out/fwd_r20.log
timeout -k 10 240 python tools/bench_forward.py --model resnet50 --batches 1,32,128,256 --iters 10 > gpurun_out/fwd_r50.log 2>&1 || exit $?
cat gpurun_out/fwd_r50.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r20 -o r20 -- python3 tools/bench_forward.py --model resnet20 --batches 1024 --iters 20 > gpurun_out/prof_r20.log 2>&1 || exit $?
echo "profile done"
