#!/bin/bash
# ResNet-50 with the strided projections fused into conv3 (OP_CONV_PROJ): GPU tests, then the
# forward A/B (GALE_FUSE_PROJ=0 vs default), 1 and 2 batches in flight, 2 interleaved rounds.
set -o pipefail
d=gpurun_out/proj
mkdir -p $d
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_bottleneck_gpu.py tests/test_models_gpu.py tests/test_kernels_gpu.py > $d/pytest.log 2>&1 \
    || { tail -30 $d/pytest.log; exit 1; }
tail -2 $d/pytest.log
: > $d/fwd_ab.jsonl
for r in 1 2; do
  for v in 0 1; do
    for f in "" "--streams 2"; do
      GALE_FUSE_PROJ=$v timeout -k 10 200 python tools/bench_forward.py --model resnet50 \
          --batches 256 --iters 30 $f | sed "s/^{/{\"fuse_proj\": $v, /" >> $d/fwd_ab.jsonl \
          || exit 1
    done
  done
done
cat $d/fwd_ab.jsonl | cut -c1-200
