#!/bin/bash
# GPU-box: kernel micro-benchmarks (JSON parser, forward) + per-kernel rocprofv3 stats.
# usage: KB_STEPS="json r50prof r20" bash tools/gpu_kbench.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in ${KB_STEPS:-json}; do
  case $step in
    json)
      timeout -k 10 180 python tools/bench_json.py > gpurun_out/kb_json.log 2>&1 || { tail -20 gpurun_out/kb_json.log; exit 1; }
      grep '^{' gpurun_out/kb_json.log ;;
    jsonprof)
      rm -rf gpurun_out/prof_json
      timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_json -o run -- \
        python3 tools/bench_json.py --batches 256 > gpurun_out/prof_json.log 2>&1 || { tail -20 gpurun_out/prof_json.log; exit 1; }
      python3 tools/prof_summary.py $(find gpurun_out/prof_json -name '*.db' | head -1) --top 8 ;;
    r20)
      timeout -k 10 180 python tools/bench_forward.py --model resnet20 --batches 256,1024,4096 > gpurun_out/kb_r20.log 2>&1 || { tail -20 gpurun_out/kb_r20.log; exit 1; }
      grep '^{' gpurun_out/kb_r20.log ;;
    r20fp8)
      timeout -k 10 180 python tools/bench_forward.py --model resnet20 --dtype fp8 --batches 256,1024,4096 > gpurun_out/kb_r20f8.log 2>&1 || { tail -20 gpurun_out/kb_r20f8.log; exit 1; }
      grep '^{' gpurun_out/kb_r20f8.log ;;
    r50)
      timeout -k 10 240 python tools/bench_forward.py --model resnet50 --batches 32,128,256 --iters 10 > gpurun_out/kb_r50.log 2>&1 || { tail -20 gpurun_out/kb_r50.log; exit 1; }
      grep '^{' gpurun_out/kb_r50.log ;;
    r50prof)
      MODEL=resnet50 PROF_CASES="bf16:256" bash tools/gpu_prof_fwd.sh || exit 1 ;;
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
# PMC pass over the JSON parser (counters from KB_PMC, one pass, <= 8 SQ counters)
if [ -n "${KB_PMC:-}" ]; then
  rm -rf gpurun_out/pmc_json
  timeout -s KILL 90 rocprofv3 --pmc ${KB_PMC} --kernel-include-regex 'json' -d gpurun_out/pmc_json -o run --output-format csv -- \
    python3 tools/bench_json.py --batches 256 --iters 5 > gpurun_out/pmc_json.log 2>&1 || { tail -20 gpurun_out/pmc_json.log; exit 1; }
  python3 tools/pmc_summary.py $(find gpurun_out/pmc_json -name '*counter_collection.csv' | head -1)
fi
for step in ${KB_STEPS2:-}; do
  case $step in
    r50paths)
      for cp in 1 0 2; do
        timeout -k 10 240 python tools/bench_forward.py --model resnet50 --batches 64,256 --iters 10 --conv-path $cp > gpurun_out/kb_r50_p$cp.log 2>&1 || { tail -20 gpurun_out/kb_r50_p$cp.log; exit 1; }
        grep '^{' gpurun_out/kb_r50_p$cp.log
      done ;;
  esac
done
