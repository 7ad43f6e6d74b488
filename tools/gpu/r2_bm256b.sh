# conv_gemm 256x128 tile with 4 waves of 128x64 (GALE_GEMM_BM256=3) vs default 128x128
set -o pipefail
mkdir -p gpurun_out
GALE_GEMM_BM256=3 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or resnet50" > gpurun_out/r2_bm256_tests3.log 2>&1 || { tail -30 gpurun_out/r2_bm256_tests3.log; exit 1; }
tail -1 gpurun_out/r2_bm256_tests3.log
for v in 0 3 0 3; do
  GALE_GEMM_BM256=$v timeout -k 10 240 python tools/bench_forward.py --model resnet50 --batches 64,256 --iters 30 > gpurun_out/r2_bm256.log 2>&1 || { tail -20 gpurun_out/r2_bm256.log; exit 1; }
  echo "BM256=$v"; grep '^{' gpurun_out/r2_bm256.log | cut -c1-200
done
