#!/bin/bash
# Round-6 evidence on ONE box (the README tables are the medians of these runs).
#   PART=a  pytest -m gpu + smoke, config 2 (headline) x3, config 3 as written x3
#   PART=b  config 1 (LeNet-5) x3, config 4 (ResNet-50, 128-image cap) x3, config 5 (fp8 and
#           bf16 with the p99 SLO controller) x2 each, interleaved
#   PART=c  kernel trace of the default bench (one hardware queue per stream under rocprofv3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r6final
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
r = json.loads(open('gpurun_out/r6final/one.jsonl').read().strip().splitlines()[-1])
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
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
        > $out/pytest_gpu.log 2>&1 || { tail -20 $out/pytest_gpu.log; exit 1; }
    tail -2 $out/pytest_gpu.log
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
    tail -1 $out/smoke.log
    for i in 1 2 3; do
      one c2_$i 240 --steps 20 --warmup 5 || exit 1
      one c3_$i 240 --steps 20 --warmup 5 --baseline-config 3 --step-images 65536 || exit 1
    done ;;
  b)
    for i in 1 2 3; do one c1_lenet5_$i 240 --model lenet5 --steps 20 --warmup 5 || exit 1; done
    for i in 1 2 3; do one c4_resnet50_$i 300 --model resnet50 --steps 10 --warmup 3 || exit 1; done
    for i in 1 2; do
      one c5_fp8_$i 240 --dtype fp8 --slo-p99-ms 2 --steps 20 --warmup 5 || exit 1
      one c5_bf16_$i 240 --slo-p99-ms 2 --steps 20 --warmup 5 || exit 1
    done ;;
  c)
    export TMPDIR=/tmp
    # one hardware queue per HIP stream under the profiler (its queue interception crashed
    # when the engine's 16 streams shared HIP's default 4, profiles/r6_e2e_kernel_stats.txt)
    GPU_MAX_HW_QUEUES=32 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        -d $out/prof -o run -- python bench.py --steps 10 --warmup 3 \
        > $out/prof_bench.log 2>&1 || { tail -20 $out/prof_bench.log; exit 1; }
    db=$(find $out/prof -name '*.db' | head -1)
    python tools/rocpd_summary.py "$db" > $out/kernel_stats.txt && head -12 $out/kernel_stats.txt ;;
esac
