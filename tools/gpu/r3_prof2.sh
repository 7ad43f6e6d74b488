#!/bin/bash
# GPU box: executor/engine GPU tests, then the default-config rocprofv3 kernel trace twice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_exec.log 2>&1 || { tail -20 gpurun_out/pytest_exec.log; exit 1; }
tail -1 gpurun_out/pytest_exec.log
bash tools/gpu/r3_prof.sh > gpurun_out/prof_run1.txt 2>&1 || { tail -40 gpurun_out/prof_run1.txt; exit 1; }
head -3 gpurun_out/prof_run1.txt
bash tools/gpu/r3_prof.sh > gpurun_out/prof_run2.txt 2>&1 || { tail -40 gpurun_out/prof_run2.txt; exit 1; }
cat gpurun_out/prof_run2.txt | head -14
