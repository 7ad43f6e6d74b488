# broker zero-copy A/B and the config-5 latency-SLO sweep (bf16 / fp8)
set -o pipefail
mkdir -p gpurun_out
for args in "--broker-zero-copy" "--no-broker-zero-copy"; do
  echo "== $args"
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 $args > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/ab.json'));print(r['value'],r['p50_latency_ms'],r['p99_latency_ms'],r['cpu_cores_busy_rank0'],r['cpu_cores_by_stage_rank0'],r['step_rate_spread'])"
done
timeout -k 10 900 python tools/slo_sweep.py --slo-ms 5 --rates 100000,200000,400000,600000,800000 --dtypes bf16,fp8 > gpurun_out/r2_slo_sweep.jsonl 2> gpurun_out/r2_slo_sweep.err || { tail -20 gpurun_out/r2_slo_sweep.err; exit 1; }
cat gpurun_out/r2_slo_sweep.jsonl
