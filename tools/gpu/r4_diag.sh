#!/bin/bash
# round-4 diagnosis: ResNet-50 with / without text pack (all engine stats); LeNet-5 latency tail
# placed in time (per-record dump + timeline)
set -o pipefail
mkdir -p gpurun_out/diag
d=gpurun_out/diag
for args in "" "--no-text-pack"; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 6 --warmup 2 --latency-load 0 --all-stats $args \
      > $d/r50.jsonl 2> $d/r50.err || { tail -5 $d/r50.err; exit 1; }
  python - "$args" <<'PY'
import json, sys
r = json.loads(open('gpurun_out/diag/r50.jsonl').read().strip().splitlines()[-1])
s = r['engine_stats_rank0']
keys = ('sparse_fetches','restored_fetches','ingested_records','records_in','batches','graph_forward_batches',
        'device_us_p50','queue_us_p50','batch_images_mean','thread_s_decode','thread_s_ingest','thread_s_submit',
        'thread_s_wait','ingest_text_bytes','ingest_link_bytes','split_records','errors')
print(repr(sys.argv[1]), r['value'], {k: s.get(k) for k in keys})
PY
done
timeout -k 10 300 python bench.py --model lenet5 --steps 20 --warmup 5 --timeline $d/tl.jsonl --timeline-ms 100 \
    --latency-dump $d/lat.npz --all-stats > $d/lenet.jsonl 2> $d/lenet.err || { tail -5 $d/lenet.err; exit 1; }
python tools/latency_report.py $d/lat.npz $d/tl.jsonl --ms 100 > $d/lenet_report.txt 2>&1
head -40 $d/lenet_report.txt | cut -c1-230
