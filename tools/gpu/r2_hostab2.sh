# host pipeline shape A/B round 2
set -o pipefail
mkdir -p gpurun_out
for args in "--partitions 8 --replicas-per-gpu 8 --decode-threads 4" "--partitions 8 --decode-threads 4" "--partitions 8 --replicas-per-gpu 8 --decode-threads 3" "--partitions 12 --replicas-per-gpu 6 --decode-threads 4" "--partitions 8 --replicas-per-gpu 4 --decode-threads 6"; do
  echo "== $args"
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 $args > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/ab.json'));print(r['value'],r['p50_latency_ms'],r['p99_latency_ms'],r['cpu_cores_busy_rank0'],r['cpu_cores_by_stage_rank0'],r['step_rate_spread'])"
done
