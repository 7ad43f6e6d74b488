#!/bin/bash
# Loopback transport cost per byte, sender + receiver, with the pipeline's 11 connections: copy
# sender (the broker's default writev) vs splice sender (zero copy), unpinned, in the GPU's NUMA
# node.
set -o pipefail
d=gpurun_out/ccd
mkdir -p $d
g++ -O2 -march=x86-64-v3 -std=c++17 -pthread -o $d/rb csrc/tests/recv_bounce_bench.cpp \
    csrc/codec/text_pack.cpp -Icsrc/include || exit 1
: > $d/rb_pairs.jsonl
for r in 1 2; do
  for s in copy splice; do
    timeout -k 5 30 taskset -c 0-63,128-191 $d/rb bounce 11 4 256 $s none >> $d/rb_pairs.jsonl || exit 1
  done
done
cat $d/rb_pairs.jsonl
