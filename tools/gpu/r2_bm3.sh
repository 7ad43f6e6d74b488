# ResNet-50 forward A/B: 3-stage 256x128 GEMM tiles (GALE_GEMM_BM256=4 when the tiles fill the chip twice, 5 whenever nkb >= 3)
set -o pipefail
mkdir -p gpurun_out
GALE_GEMM_BM256=5 timeout -k 10 200 python -u -m pytest tests/test_models_gpu.py -k "resnet50 and not fp8" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/bm3_test.log 2>&1 || { tail -30 gpurun_out/bm3_test.log; exit 1; }
tail -1 gpurun_out/bm3_test.log
for k in 0 4 5 0 4 5; do
  GALE_GEMM_BM256=$k timeout -k 10 120 python tools/bench_forward.py --model resnet50 --batches 64,256 --iters 30 > gpurun_out/bm3.log 2>&1 || { tail -20 gpurun_out/bm3.log; exit 1; }
  grep '^{' gpurun_out/bm3.log | sed "s/^{/{\"bm256\": $k, /"
done
