# SLO controller A/B on one box: backlog from unacked lag (new) vs batcher-only (old), 1.0M/1.2M offered
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, env, rate, dtype
  env $2 timeout -k 10 200 python bench.py --rate $3 --dtype $4 --steps 10 --warmup 2 --step-images 32768 --slo-p99-ms 5 > gpurun_out/sab_$1.json 2> gpurun_out/sab_$1.err || { echo FAIL $1; tail -5 gpurun_out/sab_$1.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/sab_$1.json'));print('$1',r['value'],r['record_e2e_ms_p50'],r['record_e2e_ms_p99'],r['p99_latency_ms'],r['batch_images_mean'],r['cpu_cores_busy_rank0'])"
}
run new_1m GALE_SLO_LAG_BACKLOG=1 1000000 bf16 && run old_1m GALE_SLO_LAG_BACKLOG=0 1000000 bf16 && run new_1m2 GALE_SLO_LAG_BACKLOG=1 1000000 bf16 && run old_1m2 GALE_SLO_LAG_BACKLOG=0 1000000 bf16 && run new_12 GALE_SLO_LAG_BACKLOG=1 1200000 bf16 && run old_12 GALE_SLO_LAG_BACKLOG=0 1200000 bf16 && run new_12f GALE_SLO_LAG_BACKLOG=1 1200000 fp8 && run old_12f GALE_SLO_LAG_BACKLOG=0 1200000 fp8
