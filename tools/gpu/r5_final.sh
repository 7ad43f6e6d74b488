#!/bin/bash
# Round-5 evidence on ONE box (the README tables are the medians of these runs).
#   PART=a  pytest -m gpu + smoke, config 2 (headline) x3, config 2 100-step windows x3
#   PART=b  config 1 (LeNet-5) x3, config 4 (ResNet-50) x3, placement (whole node vs 16 cores +
#           SMT siblings) x3 interleaved, world-2 shared-GPU rehearsal with and without
#           per-rank slices x2
#   PART=c  kernel trace of the default bench, forward-alone ResNet-50 / ResNet-20, ingest kernels
#   PART=d  the last code: config 2 (headline) x3 and config 4 (ResNet-50) x3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/final
mkdir -p $out
runs=$out/runs_${PART:-a}.jsonl
: > $runs

one() {  # label, seconds, bench args...
  local label=$1 secs=$2
  shift 2
  timeout -k 10 $secs python bench.py "$@" > $out/one.jsonl 2> $out/$label.err || {
    echo "FAILED $label"; tail -5 $out/$label.err; return 1; }
  python - "$label" "$runs" <<'PY'
import json, sys
r = json.loads(open('gpurun_out/final/one.jsonl').read().strip().splitlines()[-1])
r['label'] = sys.argv[1]
open(sys.argv[2], 'a').write(json.dumps(r) + '\n')
print(sys.argv[1], r['value'], 'p50', r.get('p50_latency_ms'), 'p99', r.get('p99_latency_ms'),
      'p999', r.get('p999_latency_ms'), 'dev', r['device_ms_p50'], 'cores',
      r['cpu_cores_busy_rank0'], 'spread', r['step_rate_spread']['range_pct'],
      'timed_s', r['timed_s'], flush=True)
PY
}

case ${PART:-a} in
  a)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > $out/pytest_gpu.log 2>&1 || { tail -20 $out/pytest_gpu.log; exit 1; }
    tail -2 $out/pytest_gpu.log
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
    tail -1 $out/smoke.log
    for i in 1 2 3; do one c2_$i 240 --steps 20 --warmup 5 || exit 1; done
    for i in 1 2 3; do one c2_long_$i 300 --steps 100 --warmup 5 || exit 1; done ;;
  b)
    for i in 1 2 3; do one c1_lenet5_$i 240 --model lenet5 --steps 20 --warmup 5 || exit 1; done
    for i in 1 2 3; do one c4_resnet50_$i 300 --model resnet50 --steps 10 --warmup 3 || exit 1; done
    for i in 1 2 3; do
      one node_$i 240 --steps 20 --warmup 5 || exit 1
      one smt32_$i 240 --steps 20 --warmup 5 --cpus-per-rank 32 --slice-smt || exit 1
    done
    for i in 1 2; do
      one w2_slices_$i 300 --gpus 2 --shared-gpu-rehearsal --steps 10 --warmup 3 || exit 1
      one w2_float_$i 300 --gpus 2 --shared-gpu-rehearsal --steps 10 --warmup 3 --no-rank-slices || exit 1
    done ;;
  d)
    for i in 1 2 3; do one c2_$i 240 --steps 20 --warmup 5 || exit 1; done
    for i in 1 2 3; do one c4_resnet50_$i 300 --model resnet50 --steps 10 --warmup 3 || exit 1; done ;;
  c)
    export TMPDIR=/tmp
    # one hardware queue per HIP stream under the profiler (README "--profile")
    GPU_MAX_HW_QUEUES=32 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats \
        -d $out/prof -o run -- python bench.py --steps 10 --warmup 3 --latency-load 0 \
        > $out/prof_bench.log 2>&1 || { tail -20 $out/prof_bench.log; exit 1; }
    db=$(find $out/prof -name '*.db' | head -1)
    python tools/prof_summary.py $db --top 14 > $out/kernel_stats.txt
    python tools/prof_summary.py $db --busy --top 14 > $out/kernel_busy.txt
    head -8 $out/kernel_stats.txt; cat $out/kernel_busy.txt
    rm -rf $out/prof
    timeout -k 10 240 python tools/bench_forward.py --model resnet50 --batches 64,256 --iters 30 \
        > $out/forward_resnet50.jsonl 2> $out/forward.err || exit 1
    timeout -k 10 240 python tools/bench_forward.py --model resnet50 --batches 256 --iters 30 \
        --streams 2 >> $out/forward_resnet50.jsonl 2>> $out/forward.err || exit 1
    timeout -k 10 240 python tools/bench_forward.py --model resnet20 --batches 256,4096 --iters 50 \
        > $out/forward_resnet20.jsonl 2>> $out/forward.err || exit 1
    timeout -k 10 240 python tools/bench_forward.py --model resnet20 --dtype fp8 --batches 256,4096 \
        --iters 50 >> $out/forward_resnet20.jsonl 2>> $out/forward.err || exit 1
    cat $out/forward_resnet50.jsonl $out/forward_resnet20.jsonl
    timeout -k 10 240 python tools/bench_ingest.py > $out/ingest_kernels.jsonl 2> $out/ingest.err \
        || { tail -5 $out/ingest.err; exit 1; }
    cat $out/ingest_kernels.jsonl ;;
esac
