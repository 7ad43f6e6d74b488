# same-box A/B of the host pipeline sizing: new default (12 partitions / 6 replicas / 4 decode)
# vs the previous one (4 / 4 / 2), alternated, plus the box's CPU view
set -o pipefail
mkdir -p gpurun_out
nproc; python -c "from gale.utils import host_cpus_per_rank as h; print('cpus/rank', h())"; grep -m1 "model name" /proc/cpuinfo; cat /sys/fs/cgroup/cpu.max 2>/dev/null
run() {  # tag, args
  timeout -k 10 200 python bench.py $2 > gpurun_out/sz_$1.json 2> gpurun_out/sz_$1.err || { echo FAIL $1; tail -5 gpurun_out/sz_$1.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/sz_$1.json'));print('$1',r['value'],r['p50_latency_ms'],r['cpu_cores_busy_rank0'],r['cpu_cores_by_stage_rank0'],r['step_rate_spread'])"
}
run new1 "" && run old1 "--partitions 4 --replicas-per-gpu 4 --decode-threads 2" && run new2 "" && run old2 "--partitions 4 --replicas-per-gpu 4 --decode-threads 2" && run mid1 "--partitions 8 --replicas-per-gpu 4 --decode-threads 3"
