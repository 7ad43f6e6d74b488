#!/bin/bash
# round-4 GPU step: GPU tests, 1-GPU bench A/B (default / bounce text-pack / no step graph),
# kernel trace, host receive micro-benchmark
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4_pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r4_pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r4_pytest_gpu.log | head -20; exit $rc; }
: > gpurun_out/r4_ab.jsonl
for args in "" "--text-pack" "--no-graph-step" "--text-pack" ""; do
  timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 $args > gpurun_out/r4_ab_one.jsonl 2> gpurun_out/r4_ab.err || exit 1
  python -c "
import json,sys
r=json.loads(open('gpurun_out/r4_ab_one.jsonl').read().strip().splitlines()[-1])
r['args']='$args'
print(json.dumps(r))" >> gpurun_out/r4_ab.jsonl
  python -c "
import json
r=json.loads(open('gpurun_out/r4_ab.jsonl').read().strip().splitlines()[-1])
print(r['args'], r['value'], r.get('p50_latency_ms'), r.get('p99_latency_ms'), r['link_ratio_rank0'], r['cpu_cores_busy_rank0'], r['device_ms_p50'], r['config']['path'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_prof -o run -- python bench.py --steps 10 --warmup 3 --latency-load 0 > gpurun_out/r4_prof_bench.log 2>&1 || exit 1
find gpurun_out/r4_prof -name "*kernel_stats.csv" | head -3
bash tools/gpu/r4_recv_bench.sh > /dev/null 2>&1
tail -12 gpurun_out/r4_recv_bounce_bench.jsonl
