#!/bin/bash
# Loopback receive cost per byte with the sender on the same CCD as the receiver (shared L3) vs
# another CCD vs unpinned (csrc/tests/recv_bounce_bench.cpp), copy and splice senders.
set -o pipefail
d=gpurun_out/ccd
mkdir -p $d
g++ -O2 -march=x86-64-v3 -std=c++17 -pthread -o $d/rb csrc/tests/recv_bounce_bench.cpp \
    csrc/codec/text_pack.cpp -Icsrc/include || exit 1
: > $d/rb.jsonl
for r in 1 2; do
  for snd in copy splice; do
    for pin in none same cross; do
      timeout -k 5 30 $d/rb bounce 4 4 256 $snd $pin >> $d/rb.jsonl || exit 1
    done
  done
done
cat $d/rb.jsonl
