# final check: full GPU suite, smoke, ResNet-50 forward (default conv paths), default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_pytest_gpu_full.log 2>&1 || { tail -30 gpurun_out/r2_pytest_gpu_full.log; exit 1; }
tail -1 gpurun_out/r2_pytest_gpu_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r2_smoke.log 2>&1 || { tail -20 gpurun_out/r2_smoke.log; exit 1; }
tail -1 gpurun_out/r2_smoke.log
for k in 0 1 0 1; do
  GALE_CONV_PATCH=$k timeout -k 10 120 python tools/bench_forward.py --model resnet50 --batches 256 --iters 30 > gpurun_out/fwd.log 2>&1 || { tail -20 gpurun_out/fwd.log; exit 1; }
  grep '^{' gpurun_out/fwd.log | sed "s/^{/{\"conv_patch\": $k, /" | cut -c1-160
done
timeout -k 10 240 python bench.py > gpurun_out/r2_bench_final.json 2> gpurun_out/r2_bench_final.err || { tail -20 gpurun_out/r2_bench_final.err; exit 1; }
python -c "import json;r=json.load(open('gpurun_out/r2_bench_final.json'));print(r['value'],r['timed_s'],r['p50_latency_ms'],r['p99_latency_ms'],r['cpu_cores_busy_rank0'],r['step_rate_spread'])"
