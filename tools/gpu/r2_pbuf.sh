# A/B: sink producer buffer (Kafka buffer.memory) 32 MB vs 1 GB, LeNet-5 and ResNet-20 under backlog
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, args
  timeout -k 10 300 python bench.py $2 > gpurun_out/p_$1.json 2> gpurun_out/p_$1.err || { echo FAIL $1; tail -8 gpurun_out/p_$1.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/p_$1.json'));print('$1',r['value'],r['p50_latency_ms'],r['p99_latency_ms'],r['record_e2e_ms_p50'],r['cpu_cores_by_stage_rank0'],r['step_rate_spread'])"
}
for i in 1 2; do
  run lenet_32 "--model lenet5 --producer-buffer-mb 32" && run lenet_1024 "--model lenet5 --producer-buffer-mb 1024" && \
  run r20_32 "--producer-buffer-mb 32" && run r20_1024 "--producer-buffer-mb 1024"
done
