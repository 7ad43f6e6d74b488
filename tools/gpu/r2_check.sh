# full GPU test pass + smoke + default bench + an 800k img/s open-loop run (host cores at 800k)
# + rocprof kernel stats of the bench (CRC kernel after the table change)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_pytest_gpu2.log 2>&1 || { tail -30 gpurun_out/r2_pytest_gpu2.log; exit 1; }
tail -3 gpurun_out/r2_pytest_gpu2.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r2_smoke.log 2>&1 || { tail -20 gpurun_out/r2_smoke.log; exit 1; }
tail -2 gpurun_out/r2_smoke.log
timeout -k 10 240 python bench.py > gpurun_out/r2_bench_chk.json 2> gpurun_out/r2_bench_chk.err || { tail -20 gpurun_out/r2_bench_chk.err; exit 1; }
python -c "import json;r=json.load(open('gpurun_out/r2_bench_chk.json'));print(r['value'],r['p50_latency_ms'],r['cpu_cores_busy_rank0'],r['cpu_cores_by_stage_rank0'],r['step_rate_spread'])"
timeout -k 10 240 python bench.py --rate 800000 > gpurun_out/r2_bench_800k.json 2> gpurun_out/r2_bench_800k.err || { tail -20 gpurun_out/r2_bench_800k.err; exit 1; }
python -c "import json;r=json.load(open('gpurun_out/r2_bench_800k.json'));print(r['value'],r['record_e2e_ms_p50'],r['record_e2e_ms_p99'],r['cpu_cores_busy_rank0'],r['cpu_cores_by_stage_rank0'])"
rm -rf gpurun_out/prof_chk
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_chk -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_chk.log 2>&1 || { tail -20 gpurun_out/prof_chk.log; exit 1; }
python3 tools/prof_summary.py $(find gpurun_out/prof_chk -name '*.db' | head -1) --top 12 > gpurun_out/r2_prof_chk.txt 2>&1
cat gpurun_out/r2_prof_chk.txt
