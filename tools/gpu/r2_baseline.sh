set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_bench_a.json 2> gpurun_out/r2_bench_a.err && \
timeout -k 10 180 python bench.py --steps 1000 --warmup 50 > gpurun_out/r2_bench_long.json 2> gpurun_out/r2_bench_long.err && \
timeout -k 10 180 python bench.py --steps 1000 --warmup 50 --distinct 65536 > gpurun_out/r2_bench_long_distinct.json 2> gpurun_out/r2_bench_long_distinct.err
echo rc=$?
cat gpurun_out/r2_bench_*.json
