# host pipeline sizing headroom A/B (saturated 16-CPU share): default 6 replicas / 12 partitions / 4 decode vs lighter shapes, alternating x2
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, args
  timeout -k 10 240 python bench.py $2 > gpurun_out/z_$1.json 2> gpurun_out/z_$1.err || { echo FAIL $1; tail -8 gpurun_out/z_$1.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/z_$1.json'));print('$1',r['value'],r['p99_latency_ms'],r['cpu_cores_busy_rank0'],r['step_rate_spread'])"
}
for i in 1 2; do
  run d6_12_4 "" && run d5_10_3 "--replicas-per-gpu 5 --partitions 10 --decode-threads 3" && \
  run d6_12_3 "--decode-threads 3" && run d4_12_3 "--replicas-per-gpu 4 --partitions 12 --decode-threads 3"
done
