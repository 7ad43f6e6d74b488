# exact decimal->float32 JSON parsing: GPU tests + parser throughput
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r2_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r2_pytest_gpu.log
timeout -k 10 300 python tools/bench_json.py > gpurun_out/r2_bench_json.txt 2>&1 || { tail -20 gpurun_out/r2_bench_json.txt; exit 1; }
cat gpurun_out/r2_bench_json.txt
