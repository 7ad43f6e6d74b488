#!/bin/bash
# Round-5 GPU checks on ONE box. Steps (STEPS="tests bench prof" by default, any subset):
#   tests  - pytest -m gpu over TESTS (default: all of tests/), one process
#   full   - pytest -m gpu over tests/ + smoke()
#   bench  - bench.py default config x${REPS:-2} (+ BENCH_ARGS)
#   prof   - rocprofv3 --kernel-trace --stats of a short default bench -> kernel_stats / busy
#   long   - bench.py --steps 100 x${REPS:-3} (steady-state headline windows)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/check
mkdir -p $out
runs=$out/runs${TAG:+_$TAG}.jsonl
: > $runs

one() {  # label, seconds, bench args...
  local label=$1 secs=$2
  shift 2
  timeout -k 10 $secs python bench.py "$@" $BENCH_ARGS > $out/one.jsonl 2> $out/$label.err || {
    echo "FAILED $label"; tail -5 $out/$label.err; return 1; }
  python - "$label" "$runs" <<'PY'
import json, sys
r = json.loads(open('gpurun_out/check/one.jsonl').read().strip().splitlines()[-1])
r['label'] = sys.argv[1]
open(sys.argv[2], 'a').write(json.dumps(r) + '\n')
print(sys.argv[1], r['value'], 'p50', r.get('p50_latency_ms'), 'p99', r.get('p99_latency_ms'),
      'p999', r.get('p999_latency_ms'), 'dev', r['device_ms_p50'],
      'cores', r['cpu_cores_busy_rank0'], r['cpu_cores_by_stage_rank0'],
      'spread', r['step_rate_spread']['range_pct'], 'timed_s', r['timed_s'], flush=True)
PY
}

for step in ${STEPS:-tests bench prof}; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 \
          --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
      tail -3 $out/pytest_gpu.log ;;
    full)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 \
          --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
      tail -3 $out/pytest_gpu.log
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
          > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
      tail -2 $out/smoke.log ;;
    bench)
      for i in $(seq 1 ${REPS:-2}); do one bench_$i 240 --steps 20 --warmup 5 || exit 1; done ;;
    long)
      for i in $(seq 1 ${REPS:-3}); do one long_$i 300 --steps 100 --warmup 5 || exit 1; done ;;
    prof)
      export TMPDIR=/tmp
      # one hardware queue per HIP stream under the profiler (its queue interception crashed
      # when the engine's streams shared HIP's default 4; README "--profile")
      GPU_MAX_HW_QUEUES=32 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats \
          -d $out/prof -o run -- python bench.py --steps 10 --warmup 3 --latency-load 0 \
          $BENCH_ARGS > $out/prof_bench.log 2>&1 || { tail -20 $out/prof_bench.log; exit 1; }
      db=$(find $out/prof -name '*.db' | head -1)
      python tools/prof_summary.py $db --top 14 > $out/kernel_stats.txt
      python tools/prof_summary.py $db --busy --top 14 > $out/kernel_busy.txt
      tail -1 $out/prof_bench.log | cut -c1-400
      head -12 $out/kernel_stats.txt; cat $out/kernel_busy.txt
      rm -rf $out/prof ;;
  esac
done
