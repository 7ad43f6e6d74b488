#!/bin/bash
# GPU-box: ResNet-50 (BASELINE config 4) forward throughput + per-kernel profile + a short e2e run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_forward.py --model resnet50 --batches 1,32,128,256 --iters 10 > gpurun_out/r50_fwd.log 2>&1 || { tail -5 gpurun_out/r50_fwd.log; exit 1; }
grep '^{' gpurun_out/r50_fwd.log
MODEL=resnet50 PROF_CASES="bf16:256" bash tools/gpu_prof_fwd.sh || exit 1
timeout -k 10 400 python bench.py --model resnet50 --batch 64 --replicas-per-gpu 2 --steps 20 --warmup 2 --distinct 128 > gpurun_out/r50_e2e.log 2>&1 || { tail -5 gpurun_out/r50_e2e.log; exit 1; }
tail -1 gpurun_out/r50_e2e.log
