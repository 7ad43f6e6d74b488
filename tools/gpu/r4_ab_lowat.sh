#!/bin/bash
# bounce receive x SO_RCVLOWAT: does waking the consumers per window (instead of per segment)
# cut the loopback cost on either side? ResNet-20 default bench, interleaved
set -o pipefail
d=gpurun_out/lowat
mkdir -p $d
: > $d/runs.jsonl
for r in ${REPS:-1 2}; do
for kb in ${KBS:-0 256 128}; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --recv-lowat-kb $kb > $d/one.jsonl 2> $d/err.log || { tail -5 $d/err.log; exit 1; }
  python - $kb <<'PY'
import json, sys
r = json.loads(open('gpurun_out/lowat/one.jsonl').read().strip().splitlines()[-1])
r['label'] = 'lowat_%s' % sys.argv[1]
open('gpurun_out/lowat/runs.jsonl', 'a').write(json.dumps(r) + '\n')
print(r['label'], r['value'], 'p50', r['p50_latency_ms'], 'p99', r['p99_latency_ms'],
      r['cpu_cores_by_stage_rank0'], flush=True)
PY
done
done
