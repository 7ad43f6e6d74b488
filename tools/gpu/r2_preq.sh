# A/B: produce request cap 1 MB (Kafka max.request.size, new default) vs 64 MB (previous), under backlog
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, args
  timeout -k 10 300 python bench.py $2 > gpurun_out/q_$1.json 2> gpurun_out/q_$1.err || { echo FAIL $1; tail -8 gpurun_out/q_$1.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/q_$1.json'));print('$1',r['value'],r['p50_latency_ms'],r['p99_latency_ms'],r['record_e2e_ms_p50'],r['record_e2e_ms_p99'],r['cpu_cores_by_stage_rank0'],r['step_rate_spread'])"
}
for i in 1 2; do
  run lenet_1m "--model lenet5" && run lenet_64m "--model lenet5 --producer-request-kb 65536" && \
  run r20_1m "" && run r20_64m "--producer-request-kb 65536"
done
