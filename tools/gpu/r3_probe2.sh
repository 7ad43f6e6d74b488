#!/bin/bash
# latency tail vs connections: 12 (default) / 24 input partitions (one consumer each), and a
# 2 MiB per-partition fetch cap; three 0.8-load latency phases per run, broker probes
set -o pipefail
d=gpurun_out/probe2
mkdir -p $d
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --latency-sweep 0.8 --latency-repeat 2 > $d/$tag.log 2>&1 || { tail -20 $d/$tag.log; exit 1; }
  grep '^{' $d/$tag.log | tail -1 > $d/$tag.json
  python3 -c "
import json; d=json.load(open('$d/$tag.json'))
print('$tag', d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['latency_stages_ms']['broker_source'], d['latency_broker_probes'], d['cpu_cores_by_stage_rank0'])
for x in d.get('latency_sweep', []): print('   ', x['p99_ms'], x['stages_ms']['broker_source'], x['broker_probes'], x['cg_throttled_ms'])"
}
run p12 && run p24 --partitions 24 && run p12b && run p24b --partitions 24
