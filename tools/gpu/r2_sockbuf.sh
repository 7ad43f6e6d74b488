# socket buffer sizing A/B (explicit 8 MiB vs kernel autotuning vs 32 MiB), ResNet-20 and ResNet-50
set -o pipefail
mkdir -p gpurun_out
cat /proc/sys/net/core/wmem_max /proc/sys/net/core/rmem_max /proc/sys/net/ipv4/tcp_wmem /proc/sys/net/ipv4/tcp_rmem
run() {  # tag, env, args
  env $2 timeout -k 10 300 python bench.py $3 > gpurun_out/sb_$1.json 2> gpurun_out/sb_$1.err || { echo FAIL $1; tail -8 gpurun_out/sb_$1.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/sb_$1.json'));print('$1',r['value'],r['p50_latency_ms'],r['cpu_cores_busy_rank0'],r['json_mb_per_s_rank0'],r['cpu_cores_by_stage_rank0'],r['step_rate_spread'])"
}
R50="--model resnet50 --distinct 256 --steps 10 --warmup 2 --step-images 4096"
run r20_8m GALE_SOCK_BUF=8388608 "" && run r20_auto GALE_SOCK_BUF=0 "" && run r50_8m GALE_SOCK_BUF=8388608 "$R50" && run r50_auto GALE_SOCK_BUF=0 "$R50" && run r20_8m_b GALE_SOCK_BUF=8388608 "" && run r20_auto_b GALE_SOCK_BUF=0 "" && run r50_32m GALE_SOCK_BUF=33554432 "$R50"
