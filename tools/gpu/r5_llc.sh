#!/bin/bash
# Config 2 headline with and without the L3-domain pairing of broker and source threads
# (gale/llc_pair.h), interleaved: GALE_LLC_PAIR=0 vs the default.
set -o pipefail
d=gpurun_out/llc
mkdir -p $d
: > $d/ab.jsonl
for r in 1 2 3; do
  for v in 0 1; do
    GALE_LLC_PAIR=$v timeout -k 10 240 python bench.py > $d/b.json 2> $d/b.err \
        || { tail -5 $d/b.err; exit 1; }
    tail -1 $d/b.json | sed "s/^{/{\"llc_pair\": $v, /" >> $d/ab.jsonl
    tail -1 $d/b.json | cut -c1-120
  done
done
