# ResNet-50 A/B after a conv_gemm change: tests + forward timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_r50_tests.log 2>&1 || { tail -30 gpurun_out/r2_r50_tests.log; exit 1; }
tail -1 gpurun_out/r2_r50_tests.log
timeout -k 10 240 python tools/bench_forward.py --model resnet50 --batches 64,128,256 --iters 20 > gpurun_out/r2_r50_fwd.log 2>&1 || { tail -20 gpurun_out/r2_r50_fwd.log; exit 1; }
grep '^{' gpurun_out/r2_r50_fwd.log
