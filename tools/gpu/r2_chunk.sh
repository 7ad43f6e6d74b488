# ResNet-50 forward A/B: batch chunking of the leading (56x56) layers, --chunk LAYER:N
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_models_gpu.py -k chunked -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/chunk_test.log 2>&1 || { tail -30 gpurun_out/chunk_test.log; exit 1; }
tail -1 gpurun_out/chunk_test.log
for c in "" l2.0.down:64 l2.0.down:32 l2.1.conv1:64 l2.1.conv1:32 l1.0.down:64 l2.0.down:128 ""; do
  timeout -k 10 120 python tools/bench_forward.py --model resnet50 --batches 256 --iters 30 ${c:+--chunk $c} > gpurun_out/chunk.log 2>&1 || { tail -20 gpurun_out/chunk.log; exit 1; }
  grep '^{' gpurun_out/chunk.log
done
