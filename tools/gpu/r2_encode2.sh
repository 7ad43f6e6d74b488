# GPU prediction text written straight into mapped host memory: tests + bench A/B (alternated)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_format_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_encode_tests.log 2>&1 || { tail -40 gpurun_out/r2_encode_tests.log; exit 1; }
tail -1 gpurun_out/r2_encode_tests.log
run() {  # tag, args
  timeout -k 10 200 python bench.py $2 > gpurun_out/enc_$1.json 2> gpurun_out/enc_$1.err || { echo FAIL $1; tail -5 gpurun_out/enc_$1.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/enc_$1.json'));print('$1',r['value'],r['p50_latency_ms'],r['device_ms_p50'],r['cpu_cores_busy_rank0'],r['cpu_cores_by_stage_rank0'],r['step_rate_spread'])"
}
run on1 "" && run off1 "--no-gpu-encode" && run on2 "" && run off2 "--no-gpu-encode" && run on3 "" && run off3 "--no-gpu-encode"
