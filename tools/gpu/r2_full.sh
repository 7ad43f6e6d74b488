# full GPU test suite + smoke + one default bench (round-end rehearsal)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_pytest_gpu_full.log 2>&1 || { tail -30 gpurun_out/r2_pytest_gpu_full.log; exit 1; }
tail -2 gpurun_out/r2_pytest_gpu_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r2_smoke.log 2>&1 || { tail -20 gpurun_out/r2_smoke.log; exit 1; }
tail -2 gpurun_out/r2_smoke.log
timeout -k 10 240 python bench.py > gpurun_out/r2_bench_full.json 2> gpurun_out/r2_bench_full.err || { tail -20 gpurun_out/r2_bench_full.err; exit 1; }
python -c "import json;r=json.load(open('gpurun_out/r2_bench_full.json'));print(r['value'],r['p50_latency_ms'],r['cpu_cores_busy_rank0'],r['cpu_cores_by_stage_rank0'],r['step_rate_spread'])"
