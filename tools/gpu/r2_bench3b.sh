# three driver-style runs of the default bench + a rocprofv3 kernel-stats profile of one
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench_def$i.json 2> gpurun_out/r2_bench_def$i.err || { echo BENCH_FAIL $i; tail -20 gpurun_out/r2_bench_def$i.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/r2_bench_def$i.json'));print(r['value'],r['p50_latency_ms'],r['p99_latency_ms'],r['record_e2e_ms_p50'],r['cpu_cores_busy_rank0'],r['config']['replicas_per_gpu'],r['config']['partitions'],r['step_rate_spread'])"
done
rm -rf gpurun_out/prof_e2e
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e2e -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_e2e.log 2>&1 || { tail -20 gpurun_out/prof_e2e.log; exit 1; }
python3 tools/prof_summary.py $(find gpurun_out/prof_e2e -name '*.db' | head -1) --top 12 > gpurun_out/r2_prof_e2e.txt 2>&1 || find gpurun_out/prof_e2e | head
cat gpurun_out/r2_prof_e2e.txt
