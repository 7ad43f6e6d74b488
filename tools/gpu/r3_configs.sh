#!/bin/bash
# BASELINE configurations 1, 4, 5 and the single-process split dispatch on one GPU, one bench.py
# line each (tools/gpu/r3_ab.sh format)
set -o pipefail
bash tools/gpu/r3_ab.sh gpurun_out/cfg3 \
  "lenet5|--model lenet5" \
  "r50|--model resnet50 --steps 10 --warmup 3" \
  "fp8|--dtype fp8" \
  "split2|--single-process --locality-split 2" \
  "split4|--single-process --locality-split 4"
