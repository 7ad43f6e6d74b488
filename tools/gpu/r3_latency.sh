#!/bin/bash
# latency: default bench with per-record dump + timeline, then the config-5 SLO sweep (bf16, fp8)
set -o pipefail
d=gpurun_out/lat
mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --timeline $d/tl.jsonl --timeline-ms 100 --latency-dump $d/lat.npz \
  > $d/bench.log 2>&1 || { tail -20 $d/bench.log; exit 1; }
grep '^{' $d/bench.log | tail -1 > $d/bench.jsonl
timeout -k 10 800 python tools/slo_sweep.py --slo-ms 5 --repeat 2 > $d/slo.jsonl 2> $d/slo.err || { tail -20 $d/slo.err; exit 1; }
tail -1 $d/slo.jsonl
