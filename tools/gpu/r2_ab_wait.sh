# A/B: replica wait mode (spin vs sleep-poll) and the host CRC cost
set -o pipefail
mkdir -p gpurun_out
for args in "--gpu-wait-poll-us 0" "--gpu-wait-poll-us 20" "--gpu-wait-poll-us 50" "--gpu-wait-poll-us 20 --no-check-crcs"; do
  echo "== $args"
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 $args > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/ab.json'));print(r['value'],r['p50_latency_ms'],r['p99_latency_ms'],r['cpu_cores_busy_rank0'],r['cpu_cores_by_stage_rank0'],r['step_rate_spread'])"
done
