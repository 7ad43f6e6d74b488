# three driver-style default bench runs (bench.py --steps 20 --warmup 5)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/bench3.jsonl
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
  cat gpurun_out/b.json >> gpurun_out/bench3.jsonl
  python -c "import json;r=json.load(open('gpurun_out/b.json'));print(r['value'],r['timed_s'],r['p50_latency_ms'],r['cpu_cores_busy_rank0'],r['step_rate_spread'])"
done
