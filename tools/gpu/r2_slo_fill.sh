# SLO controller A/B: full batches count as capacity-bound (GALE_SLO_FULL_BATCH=1, default) vs not
set -o pipefail
mkdir -p gpurun_out
run() {  # fill dtype rate
  GALE_SLO_FULL_BATCH=$1 timeout -k 10 240 python bench.py --rate $3 --dtype $2 --steps 10 --warmup 2 --step-images 32768 --slo-p99-ms 5 > gpurun_out/sf.json 2> gpurun_out/sf.err || { tail -10 gpurun_out/sf.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/sf.json'));print('fill=$1 $2 $3', r['value'],r['record_e2e_ms_p50'],r['record_e2e_ms_p99'],r['p99_latency_ms'],r['batch_images_mean'])"
}
for i in 1 2; do
  for f in 1 0; do
    run $f fp8 1000000 && run $f fp8 1200000 && run $f bf16 1300000
  done
done
