# ResNet-50 forward A/B: single-stage GEMM form (4 workgroups per CU) up to GALE_GEMM_SS_MAXK k-steps
set -o pipefail
mkdir -p gpurun_out
for k in 1 2 4 1 2 4; do
  GALE_GEMM_SS_MAXK=$k timeout -k 10 120 python tools/bench_forward.py --model resnet50 --batches 64,256 --iters 30 > gpurun_out/ssk.log 2>&1 || { tail -20 gpurun_out/ssk.log; exit 1; }
  grep '^{' gpurun_out/ssk.log | sed "s/^{/{\"ss_maxk\": $k, /"
done
GALE_GEMM_SS_MAXK=4 timeout -k 10 200 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ssk_test.log 2>&1 || { tail -30 gpurun_out/ssk_test.log; exit 1; }
tail -1 gpurun_out/ssk_test.log
