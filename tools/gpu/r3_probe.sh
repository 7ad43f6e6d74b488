#!/bin/bash
# broker latency-tail probes over three 0.8-load latency phases; graph replay vs direct launches
set -o pipefail
d=gpurun_out/probe
mkdir -p $d
export TMPDIR=/tmp
for v in graph no-graph; do
  timeout -k 10 300 python bench.py --$v --latency-sweep 0.8 --latency-repeat 2 > $d/$v.log 2>&1 || { tail -20 $d/$v.log; exit 1; }
  grep '^{' $d/$v.log | tail -1 > $d/$v.json
  python3 -c "
import json; d=json.load(open('$d/$v.json'))
print('$v', d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['latency_stages_ms']['broker_source'], d['latency_broker_probes'], d['cpu_cores_by_stage_rank0'], d['device_ms_p50'])
for x in d.get('latency_sweep', []): print('   ', x['p99_ms'], x['stages_ms']['broker_source'], x['broker_probes'], x['cg_throttled_ms'])"
done
