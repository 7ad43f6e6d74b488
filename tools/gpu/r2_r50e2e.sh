# ResNet-50 end to end (config 4): replicas per GPU vs micro-batch size
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, args
  timeout -k 10 300 python bench.py --model resnet50 --distinct 256 --steps 10 --warmup 2 $2 > gpurun_out/r50e_$1.json 2> gpurun_out/r50e_$1.err || { echo FAIL $1; tail -8 gpurun_out/r50e_$1.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/r50e_$1.json'));print('$1',r['value'],r['p50_latency_ms'],r['device_ms_p50'],r['batch_images_mean'],r['cpu_cores_busy_rank0'],r['json_mb_per_s_rank0'],r['step_rate_spread'])"
}
run r1b256 "--replicas-per-gpu 1 --batch 256 --step-images 4096" && run r2b256 "--replicas-per-gpu 2 --batch 256 --step-images 4096" && run r2b128 "--replicas-per-gpu 2 --batch 128 --step-images 4096" && run r3b128 "--replicas-per-gpu 3 --batch 128 --step-images 4096" && run r2b256w "--replicas-per-gpu 2 --batch 256 --step-images 4096 --max-wait-us 10000"
