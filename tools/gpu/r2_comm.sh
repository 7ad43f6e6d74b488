# RCCL comm + locality refactor: GPU tests, bench (both modes at N=1), JSON parser bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r2_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r2_pytest_gpu.log
for args in "" "--single-process" ""; do
  echo "== $args"
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 $args > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/ab.json'));print(r['value'],r['p50_latency_ms'],r['p99_latency_ms'],r['cpu_cores_busy_rank0'],r['cpu_cores_by_stage_rank0'],r['step_rate_spread'])"
done
timeout -k 10 300 python tools/bench_json.py > gpurun_out/r2_bench_json.txt 2>&1 || { tail -20 gpurun_out/r2_bench_json.txt; exit 1; }
cat gpurun_out/r2_bench_json.txt
