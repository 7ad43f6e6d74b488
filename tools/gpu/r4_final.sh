#!/bin/bash
# Round-4 evidence on ONE box: every BASELINE config 3 runs back to back (the README tables are
# the medians of these), GPU tests + smoke, the plain multi-GPU entry point, a kernel trace.
#   PART=a  pytest -m gpu, smoke, config 2 (ResNet-20 bf16) x3, config 1 (LeNet-5) x3
#   PART=b  config 5 (p99 SLO 2 ms) fp8 x3 and bf16 x3, config 4 (ResNet-50) x3,
#           bench.py --gpus 2 (rehearsal / refusal),
#           kernel trace of the default bench, forward-alone ResNet-50 / ResNet-20
#   PART=c  only the kernel trace and the forward-alone runs
#   PART=b2 config 4 x3, then PART=c
#   PART=b5 config 5 only
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
      'dev', r['device_ms_p50'], 'cores', r['cpu_cores_busy_rank0'],
      'spread', r['step_rate_spread']['range_pct'], flush=True)
PY
}

if [ "${PART:-a}" = a ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > $out/pytest_gpu.log 2>&1 || { tail -20 $out/pytest_gpu.log; exit 1; }
  tail -2 $out/pytest_gpu.log
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
      > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
  tail -1 $out/smoke.log
  for i in 1 2 3; do one c2_bf16_$i 240 --steps 20 --warmup 5 || exit 1; done
  for i in 1 2 3; do one c1_lenet5_$i 240 --model lenet5 --steps 20 --warmup 5 || exit 1; done
elif [ "$PART" = b ]; then
  for i in 1 2 3; do  # fp8 and bf16 interleaved
    one c5_fp8_slo2_$i 240 --steps 20 --warmup 5 --dtype fp8 --slo-p99-ms 2 || exit 1
    one c5_bf16_slo2_$i 240 --steps 20 --warmup 5 --slo-p99-ms 2 || exit 1
  done
  for i in 1 2 3; do one c4_resnet50_$i 300 --model resnet50 --steps 10 --warmup 3 || exit 1; done
  # the driver's multi-GPU entry point on a 1-GPU box: more ranks than GPUs must be refused,
  # and the same entry point with --shared-gpu-rehearsal runs both ranks (gloo, one GPU)
  if timeout -k 10 120 python bench.py --gpus 2 --steps 2 --warmup 1 > $out/gpus2_refused.log 2>&1; then
    echo "bench.py --gpus 2 did not fail on a 1-GPU box"; exit 1
  fi
  tail -2 $out/gpus2_refused.log
  one rehearsal_world2 300 --gpus 2 --shared-gpu-rehearsal --steps 10 --warmup 3 || exit 1
elif [ "$PART" = c1 ]; then
  for i in 1 2 3; do one c1_lenet5_$i 240 --model lenet5 --steps 20 --warmup 5 || exit 1; done
elif [ "$PART" = b5 ]; then
  for i in 1 2 3; do  # fp8 and bf16 interleaved
    one c5_fp8_slo2_$i 240 --steps 20 --warmup 5 --dtype fp8 --slo-p99-ms 2 || exit 1
    one c5_bf16_slo2_$i 240 --steps 20 --warmup 5 --slo-p99-ms 2 || exit 1
  done
elif [ "$PART" = b2 ]; then
  for i in 1 2 3; do one c4_resnet50_$i 300 --model resnet50 --steps 10 --warmup 3 || exit 1; done
fi
if [ "${PART:-a}" = b ] || [ "${PART:-a}" = c ] || [ "${PART:-a}" = b2 ]; then
  export TMPDIR=/tmp
  # one hardware queue per HIP stream under the profiler: its queue interception crashed when
  # the engine's streams (replicas + ingest lanes, > 4 from several threads) shared HIP's
  # default 4 (a SIGSEGV inside librocprofiler-sdk under GpuIngest::run,
  # gpurun_out/final/prof_bench.log); the same setting gale's --profile uses
  export GPU_MAX_HW_QUEUES=32
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- \
      python bench.py --steps 10 --warmup 3 --latency-load 0 > $out/prof_bench.log 2>&1 || exit 1
  db=$(find $out/prof -name '*.db' | head -1)
  python tools/prof_summary.py $db --top 14 > $out/kernel_stats.txt
  python tools/prof_summary.py $db --busy --top 14 > $out/kernel_busy.txt
  head -8 $out/kernel_stats.txt; cat $out/kernel_busy.txt
  rm -rf $out/prof  # (the trace database: too large to bring back)
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
  cat $out/ingest_kernels.jsonl
fi
