# BASELINE configs 1, 2, 4 (fp32 plan too) end to end on 1 GPU with the session's final code
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, args
  timeout -k 10 300 python bench.py $2 > gpurun_out/cfg_$1.json 2> gpurun_out/cfg_$1.err || { echo FAIL $1; tail -8 gpurun_out/cfg_$1.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/cfg_$1.json'));print('$1',r['value'],r['timed_s'],r['p50_latency_ms'],r['record_e2e_ms_p99'],r['batch_images_mean'],r['cpu_cores_busy_rank0'],r['json_mb_per_s_rank0'],r['step_rate_spread'])"
}
run lenet5 "--model lenet5 --steps 20 --warmup 5" && \
run r20_bf16 "--steps 20 --warmup 5" && \
run r20_fp8 "--dtype fp8 --steps 20 --warmup 5" && \
run r20_fp32 "--dtype fp32 --steps 20 --warmup 5" && \
run r50_b256 "--model resnet50 --batch 256 --step-images 4096 --distinct 256 --steps 10 --warmup 2"
cat gpurun_out/cfg_*.json > gpurun_out/configs_final.jsonl
