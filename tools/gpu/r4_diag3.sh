#!/bin/bash
# ResNet-50 with the text pack: why do records miss the GPU ingest (pinned-pool counters)
set -o pipefail
d=gpurun_out/diag3
mkdir -p $d
for mode in pack nopack; do
  extra=""; [ $mode = nopack ] && extra="--no-text-pack"
  timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 --all-stats $extra \
    > $d/$mode.jsonl 2> $d/$mode.err || { tail -5 $d/$mode.err; exit 1; }
  python - $d/$mode.jsonl $mode <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = r['engine_stats_rank0']
print(sys.argv[2], r['value'], r['device_ms_p50'], r['cpu_cores_busy_rank0'],
      {k: v for k, v in s.items() if k.startswith('pinned') or k in ('ingested_records', 'records_in', 'sparse_fetches', 'restored_fetches', 'queue_records')})
PY
  grep -i "gale\|error\|fail" $d/$mode.err | head -5 || true
done
