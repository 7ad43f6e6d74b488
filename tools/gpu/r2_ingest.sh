# GPU ingest: tests, then bench with/without device-side CRC + image counting
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r2_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r2_pytest_gpu.log
for args in "--gpu-ingest" "--no-gpu-ingest" "--gpu-ingest --gpu-wait-poll-us 20" "--gpu-ingest"; do
  echo "== $args"
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 $args > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/ab.json'));print(r['value'],r['p50_latency_ms'],r['p99_latency_ms'],r['cpu_cores_busy_rank0'],r['cpu_cores_by_stage_rank0'],r['step_rate_spread'])"
done
