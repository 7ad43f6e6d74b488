#!/bin/bash
# decode (GPU-ingest) threads x replicas per GPU with the 10 source threads, ResNet-20 defaults,
# interleaved x2
set -o pipefail
d=gpurun_out/threads
mkdir -p $d
: > $d/runs.jsonl
for r in 1 2; do
for v in "d6r6|" "d4r6|--decode-threads 4" "d6r4|--replicas-per-gpu 4" "d4r4|--decode-threads 4 --replicas-per-gpu 4"; do
  label=${v%%|*}; args=${v#*|}
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 $args > $d/one.jsonl 2> $d/err.log || { tail -5 $d/err.log; exit 1; }
  python - $label <<'PY'
import json, sys
r = json.loads(open('gpurun_out/threads/one.jsonl').read().strip().splitlines()[-1])
r['label'] = sys.argv[1]
open('gpurun_out/threads/runs.jsonl', 'a').write(json.dumps(r) + '\n')
print(r['label'], r['value'], 'p50', r['p50_latency_ms'], 'p99', r['p99_latency_ms'],
      r['cpu_cores_by_stage_rank0'], flush=True)
PY
done
done
