#!/bin/bash
# round-4 A/B: bounce window sizes, then the other BASELINE configs with the new defaults
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r4_ab2.jsonl
: > $out
run() {  # $1 = label, rest = bench args
  local label=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" > gpurun_out/r4_one.jsonl 2> gpurun_out/r4_one.err || { tail -5 gpurun_out/r4_one.err; return 1; }
  python - "$label" <<'PY'
import json, sys
r = json.loads(open('gpurun_out/r4_one.jsonl').read().strip().splitlines()[-1])
r['label'] = sys.argv[1]
open('gpurun_out/r4_ab2.jsonl', 'a').write(json.dumps(r) + '\n')
print(sys.argv[1], r['value'], r.get('p50_latency_ms'), r.get('p99_latency_ms'), r['link_ratio_rank0'],
      r['cpu_cores_busy_rank0'], r['cpu_cores_by_stage_rank0'], r['step_rate_spread']['range_pct'])
PY
}
run default --steps 20 --warmup 5 || exit 1
run win1024 --steps 20 --warmup 5 --text-pack-window-kb 1024 || exit 1
run win64 --steps 20 --warmup 5 --text-pack-window-kb 64 || exit 1
run nopack --steps 20 --warmup 5 --no-text-pack || exit 1
run default --steps 20 --warmup 5 || exit 1
run lenet5 --model lenet5 --steps 20 --warmup 5 || exit 1
run resnet50 --model resnet50 --steps 10 --warmup 3 || exit 1
run fp8_slo2 --dtype fp8 --slo-p99-ms 2 --steps 20 --warmup 5 --latency-sweep 0.6,0.8,0.9 || exit 1
