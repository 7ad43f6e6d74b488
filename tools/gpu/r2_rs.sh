# ResNet-50 forward A/B: register-staged GEMM tiles (GALE_GEMM_RS: 0 LDS-DMA, 1 k-loop, 2 + K=64 form, 3 + stem)
set -o pipefail
mkdir -p gpurun_out
GALE_GEMM_RS=3 timeout -k 10 200 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/rs_test.log 2>&1 || { tail -30 gpurun_out/rs_test.log; exit 1; }
tail -1 gpurun_out/rs_test.log
for k in 0 1 2 3 0 1 2 3; do
  GALE_GEMM_RS=$k timeout -k 10 120 python tools/bench_forward.py --model resnet50 --batches 64,256 --iters 30 > gpurun_out/rs.log 2>&1 || { tail -20 gpurun_out/rs.log; exit 1; }
  grep '^{' gpurun_out/rs.log | sed "s/^{/{\"rs\": $k, /" | cut -c1-140
done
