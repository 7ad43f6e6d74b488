# LeNet-5 end to end at fixed offered loads (is the ~1 s backlog p50 queueing or a stall?)
set -o pipefail
mkdir -p gpurun_out
for r in 500000 1000000 1500000; do
  timeout -k 10 300 python bench.py --model lenet5 --rate $r --steps 10 --warmup 2 > gpurun_out/lr.json 2> gpurun_out/lr.err || { tail -8 gpurun_out/lr.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/lr.json'));print($r, r['value'],r['p50_latency_ms'],r['p99_latency_ms'],r['record_e2e_ms_p50'],r['record_e2e_ms_p99'],r['device_ms_p50'],r['batch_images_mean'],r['cpu_cores_by_stage_rank0'])"
done
