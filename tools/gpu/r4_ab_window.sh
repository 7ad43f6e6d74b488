#!/bin/bash
# bounce window size with the window-sized receive low-water mark (the default since
# profiles/r4_ab_recv_lowat.jsonl), ResNet-20 defaults, interleaved; plus the box's socket limits
set -o pipefail
d=gpurun_out/window
mkdir -p $d
cat /proc/sys/net/core/rmem_max /proc/sys/net/core/wmem_max /proc/sys/net/ipv4/tcp_rmem > $d/sysctl.txt 2>&1
cat $d/sysctl.txt
: > $d/runs.jsonl
for r in 1 2; do
for kb in 256 512 1024; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --text-pack-window-kb $kb > $d/one.jsonl 2> $d/err.log || { tail -5 $d/err.log; exit 1; }
  python - $kb <<'PY'
import json, sys
r = json.loads(open('gpurun_out/window/one.jsonl').read().strip().splitlines()[-1])
r['label'] = 'window_%s' % sys.argv[1]
open('gpurun_out/window/runs.jsonl', 'a').write(json.dumps(r) + '\n')
print(r['label'], r['value'], 'p50', r['p50_latency_ms'], 'p99', r['p99_latency_ms'],
      r['cpu_cores_by_stage_rank0'], flush=True)
PY
done
done
