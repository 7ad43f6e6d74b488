#!/bin/bash
# round-4 GPU check: GPU tests, 1-GPU bench, the plain multi-rank entry point (shared-GPU
# rehearsal) and the loud failure for more GPUs than the box has
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4_pytest_gpu.log 2>&1 && tail -3 gpurun_out/r4_pytest_gpu.log &&
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_bench1.jsonl 2> gpurun_out/r4_bench1.err &&
tail -c 600 gpurun_out/r4_bench1.jsonl &&
timeout -k 10 240 python bench.py --gpus 2 --shared-gpu-rehearsal --steps 10 --warmup 3 \
    --latency-load 0 > gpurun_out/r4_rehearsal2.jsonl 2> gpurun_out/r4_rehearsal2.err &&
tail -c 600 gpurun_out/r4_rehearsal2.jsonl
rc=$?
echo "chain rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 60 python bench.py --gpus 2 --steps 1 > gpurun_out/r4_gpus2_fail.log 2>&1
echo "bench --gpus 2 on a 1-GPU box: rc=$?"; cat gpurun_out/r4_gpus2_fail.log | tail -2
exit $rc
