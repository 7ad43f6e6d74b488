# ResNet-50 conv_gemm 3-stage ring A/B (GALE_GEMM_RING) + kernel/model tests + per-layer timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_ring_tests.log 2>&1 || { tail -30 gpurun_out/r2_ring_tests.log; exit 1; }
tail -1 gpurun_out/r2_ring_tests.log
for v in GALE_GEMM_RING=0 GALE_GEMM_RING=1 GALE_GEMM_RING=0 GALE_GEMM_RING=1; do
  env $v timeout -k 10 240 python tools/bench_forward.py --model resnet50 --batches 64,256 --iters 30 > gpurun_out/r2_r50_ring.log 2>&1 || { tail -20 gpurun_out/r2_r50_ring.log; exit 1; }
  echo "$v"; grep '^{' gpurun_out/r2_r50_ring.log
done
