#!/bin/bash
# conv_gemm with three LDS stages (GALE_CONV_STAGES=3: two k-steps of DMA in flight, one
# workgroup per CU) vs two (default): single-layer times (tools/bench_conv.py, batch 256 and
# 128), the ResNet-50 forward (tools/bench_forward.py), and the model numerics under the
# three-stage form.
# (The three-stage form was not kept: GALE_CONV_STAGES no longer exists, both arms now run the
# same code. Results: profiles/r6_conv_stages_ab.jsonl.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r6s
mkdir -p $out
for i in 1 2; do
  for s in 2 3; do
    for b in 256 128; do
      GALE_CONV_STAGES=$s timeout -k 10 120 python tools/bench_conv.py --batch $b --tag s${s}_b${b}_$i \
          >> $out/conv.jsonl 2> $out/conv.err || { tail -5 $out/conv.err; exit 1; }
    done
    GALE_CONV_STAGES=$s timeout -k 10 180 python tools/bench_forward.py --model resnet50 \
        --batches 128,256 --iters 20 > $out/fwd_s${s}_$i.log 2>&1 || { tail -5 $out/fwd_s${s}_$i.log; exit 1; }
    tail -2 $out/fwd_s${s}_$i.log
  done
done
cat $out/conv.jsonl
GALE_CONV_STAGES=3 timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -q -k resnet50 \
    --timeout 240 --timeout-method thread > $out/pytest_s3.log 2>&1; tail -2 $out/pytest_s3.log
