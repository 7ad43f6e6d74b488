# fp8 / LeNet end-to-end diagnosis: per-step rates and stage cores
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, args
  timeout -k 10 300 python bench.py $2 > gpurun_out/d_$1.json 2> gpurun_out/d_$1.err || { echo FAIL $1; tail -8 gpurun_out/d_$1.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/d_$1.json'));print('$1',r['value'],r['p50_latency_ms'],r['device_ms_p50'],r['batch_images_mean'],r['cpu_cores_by_stage_rank0']);print(r['step_rates'])"
}
run fp8a "--dtype fp8" && run bf16 "" && run fp8b "--dtype fp8 --no-gpu-encode" && run lenet "--model lenet5"
