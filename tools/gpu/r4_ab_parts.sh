#!/bin/bash
# input partitions (= source threads) per GPU, 12 default, ResNet-20
# defaults, interleaved
set -o pipefail
d=gpurun_out/parts
mkdir -p $d
: > $d/runs.jsonl
for r in ${REPS:-1 2}; do
for us in ${VALS:-12 16 8}; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --partitions $us > $d/one.jsonl 2> $d/err.log || { tail -5 $d/err.log; exit 1; }
  python - $us <<'PY'
import json, sys
r = json.loads(open('gpurun_out/parts/one.jsonl').read().strip().splitlines()[-1])
r['label'] = 'parts_%s' % sys.argv[1]
open('gpurun_out/parts/runs.jsonl', 'a').write(json.dumps(r) + '\n')
print(r['label'], r['value'], 'p50', r['p50_latency_ms'], 'p99', r['p99_latency_ms'],
      r['cpu_cores_by_stage_rank0'], flush=True)
PY
done
done
