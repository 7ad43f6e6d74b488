# fp8 at 1.0 M offered: SLO controller on vs off (is the controller's limit cycle the cause?)
set -o pipefail
mkdir -p gpurun_out
for slo in 5 0 5 0; do
  timeout -k 10 240 python bench.py --rate 1000000 --dtype fp8 --steps 10 --warmup 2 --step-images 32768 --slo-p99-ms $slo > gpurun_out/f8.json 2> gpurun_out/f8.err || { tail -10 gpurun_out/f8.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/f8.json'));print('slo=$slo', r['value'],r['record_e2e_ms_p50'],r['record_e2e_ms_p99'],r['p99_latency_ms'],r['batch_images_mean'],r['step_rates'])"
done
