# A/B at the current default sizing: broker zero-copy fetch sends (vmsplice+splice) on / off, alternating
set -o pipefail
mkdir -p gpurun_out
for args in "--broker-zero-copy" "--no-broker-zero-copy" "--broker-zero-copy" "--no-broker-zero-copy" "--broker-zero-copy" "--no-broker-zero-copy"; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 $args > gpurun_out/zc.json 2> gpurun_out/zc.err || { tail -20 gpurun_out/zc.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/zc.json'));print('$args', r['value'],r['p50_latency_ms'],r['cpu_cores_busy_rank0'],r['cpu_cores_by_stage_rank0'],r['step_rate_spread'])"
done
