#!/bin/bash
# sleep-poll interval of the replica (and GPU-ingest) completion waits, 20 us default, ResNet-20
# defaults, interleaved
set -o pipefail
d=gpurun_out/poll
mkdir -p $d
: > $d/runs.jsonl
for r in 1 2; do
for us in 20 60 150; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --gpu-wait-poll-us $us > $d/one.jsonl 2> $d/err.log || { tail -5 $d/err.log; exit 1; }
  python - $us <<'PY'
import json, sys
r = json.loads(open('gpurun_out/poll/one.jsonl').read().strip().splitlines()[-1])
r['label'] = 'poll_%s' % sys.argv[1]
open('gpurun_out/poll/runs.jsonl', 'a').write(json.dumps(r) + '\n')
print(r['label'], r['value'], 'p50', r['p50_latency_ms'], 'p99', r['p99_latency_ms'],
      r['cpu_cores_by_stage_rank0'], flush=True)
PY
done
done
