#!/bin/bash
# input partitions (= consumer connections) per GPU: 12 vs 24 (vs 16), alternating, default bench
set -o pipefail
d=gpurun_out/partsab
mkdir -p $d
export TMPDIR=/tmp
for i in 1 2 3; do
  for p in 12 24 16; do
    timeout -k 10 300 python bench.py --partitions $p --latency-sweep 0.8 > $d/p${p}_$i.log 2>&1 || { tail -20 $d/p${p}_$i.log; exit 1; }
    grep '^{' $d/p${p}_$i.log | tail -1 > $d/p${p}_$i.json
    python3 -c "
import json; d=json.load(open('$d/p${p}_$i.json'))
print($p, $i, d['value'], d['step_rate_spread']['range_pct'], d['p50_latency_ms'], d['p99_latency_ms'], [x['p99_ms'] for x in d.get('latency_sweep', [])], d['cpu_cores_busy_rank0'], d['latency_broker_probes']['flush_slow'])"
  done
done
