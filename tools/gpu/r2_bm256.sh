# conv_gemm 256x128 tiles (GALE_GEMM_BM256 0 off / 2 by size / 1 always) A/B + tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_bm256_tests.log 2>&1 || { tail -30 gpurun_out/r2_bm256_tests.log; exit 1; }
tail -1 gpurun_out/r2_bm256_tests.log
GALE_GEMM_BM256=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or resnet50" > gpurun_out/r2_bm256_tests1.log 2>&1 || { tail -30 gpurun_out/r2_bm256_tests1.log; exit 1; }
tail -1 gpurun_out/r2_bm256_tests1.log
for v in 0 2 1 0 2 1; do
  GALE_GEMM_BM256=$v timeout -k 10 240 python tools/bench_forward.py --model resnet50 --batches 64,256 --iters 30 > gpurun_out/r2_bm256.log 2>&1 || { tail -20 gpurun_out/r2_bm256.log; exit 1; }
  echo "BM256=$v"; grep '^{' gpurun_out/r2_bm256.log | cut -c1-200
done
