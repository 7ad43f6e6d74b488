# BASELINE configs 1 (LeNet-5) and 4 (ResNet-50 224x224x3 records) end to end on 1 GPU
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, args
  timeout -k 10 300 python bench.py $2 > gpurun_out/cfg_$1.json 2> gpurun_out/cfg_$1.err || { echo FAIL $1; tail -8 gpurun_out/cfg_$1.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/cfg_$1.json'));print('$1',r['value'],r['p50_latency_ms'],r['device_ms_p50'],r['batch_images_mean'],r['cpu_cores_busy_rank0'],r['json_mb_per_s_rank0'],r['cpu_cores_by_stage_rank0'],r['step_rate_spread'])"
}
run lenet5 "--model lenet5 --steps 20 --warmup 5" && run r50_b64 "--model resnet50 --batch 64 --step-images 2048 --distinct 256 --steps 10 --warmup 2" && run r50_b256 "--model resnet50 --batch 256 --step-images 4096 --distinct 256 --steps 10 --warmup 2"
