# fp32 reference-precision plan: kernel + model tests, then all GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q -s -k "f32 or fp32" --timeout 120 --timeout-method thread > gpurun_out/r2_fp32.log 2>&1; rc=$?
grep -E "fp32 plan|passed|failed|Error|error" gpurun_out/r2_fp32.log | head -30
[ $rc -eq 0 ] || { tail -30 gpurun_out/r2_fp32.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r2_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r2_pytest_gpu.log
timeout -k 10 240 python bench.py --steps 5 --warmup 2 --dtype fp32 --min-warmup-s 1 > gpurun_out/r2_bench_fp32.json 2> gpurun_out/r2_bench_fp32.err || { tail -20 gpurun_out/r2_bench_fp32.err; exit 1; }
cat gpurun_out/r2_bench_fp32.json
