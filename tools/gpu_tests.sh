#!/bin/bash
# GPU-box: the full GPU test suite in ONE pytest process (stops at the first failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
exit $rc
