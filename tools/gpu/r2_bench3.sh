# round 2: GPU tests, then three driver-style steady-state bench runs (spread across runs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r2_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r2_pytest_gpu.log
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench_run$i.json 2> gpurun_out/r2_bench_run$i.err || { echo BENCH_FAIL $i; tail -20 gpurun_out/r2_bench_run$i.err; exit 1; }
  cat gpurun_out/r2_bench_run$i.json
done
