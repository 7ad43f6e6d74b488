# ResNet-50 e2e: many fetch partitions, few replicas, longer batching window (bigger batches)
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, args
  timeout -k 10 300 python bench.py --model resnet50 --distinct 256 --steps 10 --warmup 2 --step-images 4096 --batch 256 $2 > gpurun_out/r50g_$1.json 2> gpurun_out/r50g_$1.err || { echo FAIL $1; tail -8 gpurun_out/r50g_$1.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/r50g_$1.json'));print('$1',r['value'],r['p50_latency_ms'],r['device_ms_p50'],r['batch_images_mean'],r['cpu_cores_busy_rank0'],r['json_mb_per_s_rank0'],r['step_rate_spread'])"
}
run r2p12w10 "--replicas-per-gpu 2 --partitions 12 --max-wait-us 10000" && run r2p12w20 "--replicas-per-gpu 2 --partitions 12 --max-wait-us 20000" && run r1p12w20 "--replicas-per-gpu 1 --partitions 12 --max-wait-us 20000" && run r3p12w20 "--replicas-per-gpu 3 --partitions 12 --max-wait-us 20000" && run r2p16w20 "--replicas-per-gpu 2 --partitions 16 --max-wait-us 20000"
