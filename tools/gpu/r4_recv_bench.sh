#!/bin/bash
# host receive-path micro-benchmark on the GPU box's CPU (csrc/tests/recv_bounce_bench.cpp)
set -o pipefail
mkdir -p gpurun_out
g++ -O3 -std=c++17 -march=native -pthread csrc/tests/recv_bounce_bench.cpp csrc/codec/text_pack.cpp \
    -o /tmp/recv_bounce_bench || exit 1
out=gpurun_out/r4_recv_bounce_bench.jsonl
: > $out
for pairs in 1 4 8; do
  for m in raw pack2 bounce; do
    timeout -k 5 20 /tmp/recv_bounce_bench $m $pairs 3 256 | tee -a $out
  done
done
for piece in 64 1024; do
  timeout -k 5 20 /tmp/recv_bounce_bench bounce 4 3 $piece | tee -a $out
done
lscpu | grep -E "Model name|L2|L3" >> $out
