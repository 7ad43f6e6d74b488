#!/bin/bash
# confirm: ResNet-50 with the doubled pinned budget for packed chunks; LeNet-5 tail with the chunked
# ack log; ResNet-20 default
set -o pipefail
mkdir -p gpurun_out/diag2
d=gpurun_out/diag2
: > $d/runs.jsonl
for spec in "resnet50|--model resnet50 --steps 10 --warmup 3" "lenet5|--model lenet5 --steps 20 --warmup 5" "resnet20|--steps 20 --warmup 5"; do
  label=${spec%%|*}; args=${spec#*|}
  timeout -k 10 300 python bench.py $args --all-stats > $d/one.jsonl 2> $d/one.err || { tail -5 $d/one.err; exit 1; }
  python - "$label" <<'PY'
import json, sys
r = json.loads(open('gpurun_out/diag2/one.jsonl').read().strip().splitlines()[-1])
r['label'] = sys.argv[1]
open('gpurun_out/diag2/runs.jsonl', 'a').write(json.dumps(r) + '\n')
s = r['engine_stats_rank0']
print(sys.argv[1], r['value'], r.get('p50_latency_ms'), r.get('p99_latency_ms'), r['device_ms_p50'],
      r['cpu_cores_busy_rank0'], r['step_rate_spread']['range_pct'], r.get('latency_stages_ms'),
      {k: s.get(k) for k in ('ingested_records', 'records_in', 'sparse_fetches')})
PY
done
