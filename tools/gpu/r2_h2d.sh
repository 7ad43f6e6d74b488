# pinned H2D bandwidth + ResNet-50 e2e with many fetch partitions but few big-batch replicas
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/h2d_bw.py
run() {  # tag, args
  timeout -k 10 300 python bench.py --model resnet50 --distinct 256 --steps 10 --warmup 2 --step-images 4096 $2 > gpurun_out/r50f_$1.json 2> gpurun_out/r50f_$1.err || { echo FAIL $1; tail -8 gpurun_out/r50f_$1.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/r50f_$1.json'));print('$1',r['value'],r['p50_latency_ms'],r['device_ms_p50'],r['batch_images_mean'],r['cpu_cores_busy_rank0'],r['json_mb_per_s_rank0'],r['step_rate_spread'])"
}
run r2p12 "--replicas-per-gpu 2 --partitions 12 --batch 256 --max-wait-us 5000" && run r3p12 "--replicas-per-gpu 3 --partitions 12 --batch 256 --max-wait-us 5000" && run r2p16 "--replicas-per-gpu 2 --partitions 16 --decode-threads 6 --batch 256 --max-wait-us 5000"
