#!/bin/bash
# After the ingest counting fix + high-priority ingest streams: ResNet-50 with / without the text
# pack (interleaved), with the pool counters; ResNet-20 default for the headline path
set -o pipefail
d=gpurun_out/diag5
mkdir -p $d
: > $d/runs.jsonl
for spec in "r50_pack|--model resnet50 --steps 10 --warmup 3" \
            "r50_nopack|--model resnet50 --steps 10 --warmup 3 --no-text-pack" \
            "r50_pack|--model resnet50 --steps 10 --warmup 3" \
            "r50_nopack|--model resnet50 --steps 10 --warmup 3 --no-text-pack" \
            "r20|--steps 20 --warmup 5" "r20|--steps 20 --warmup 5"; do
  label=${spec%%|*}; args=${spec#*|}
  timeout -k 10 300 python bench.py $args --all-stats > $d/one.jsonl 2> $d/$label.err || { tail -5 $d/$label.err; exit 1; }
  python - "$label" <<'PY'
import json, sys
r = json.loads(open('gpurun_out/diag5/one.jsonl').read().strip().splitlines()[-1])
r['label'] = sys.argv[1]
open('gpurun_out/diag5/runs.jsonl', 'a').write(json.dumps(r) + '\n')
s = r['engine_stats_rank0']
print(sys.argv[1], r['value'], 'p50', r.get('p50_latency_ms'), 'p99', r.get('p99_latency_ms'),
      'dev', r['device_ms_p50'], 'cores', r['cpu_cores_busy_rank0'],
      'spread', r['step_rate_spread']['range_pct'], {k: s.get(k) for k in (
          'pinned_chunks', 'pinned_waits', 'pinned_wait_s', 'pinned_heap_budget',
          'queue_records', 'thread_s_ingest', 'batch_images_mean')}, flush=True)
PY
done
