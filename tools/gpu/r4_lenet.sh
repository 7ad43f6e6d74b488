#!/bin/bash
# BASELINE config 1 (LeNet-5) x3 with the 1 M-image steps, latency at 0.9 x load
set -o pipefail
d=gpurun_out/lenet
mkdir -p $d
: > $d/runs.jsonl
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --model lenet5 --steps 20 --warmup 5 --latency-load 0.9 \
      > $d/one.jsonl 2> $d/err_$i.log || { tail -5 $d/err_$i.log; exit 1; }
  python - $i <<'PY'
import json, sys
r = json.loads(open('gpurun_out/lenet/one.jsonl').read().strip().splitlines()[-1])
r['label'] = 'c1_lenet5_%s' % sys.argv[1]
open('gpurun_out/lenet/runs.jsonl', 'a').write(json.dumps(r) + '\n')
print(r['label'], r['value'], 'p50', r['p50_latency_ms'], 'p99', r['p99_latency_ms'], 'offered',
      r['latency_offered_img_s'], 'spread', r['step_rate_spread']['range_pct'], 'timed_s',
      r['timed_s'], r.get('timed_cgroup_rank0'), flush=True)
PY
done
