#!/bin/bash
# round-4 A/B 3: ResNet-50 (config 4) text pack on/off + kernel trace; LeNet-5 (config 1) sink
# parallelism / producer buffer
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r4_ab3.jsonl
run() {
  local label=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" > gpurun_out/r4_one.jsonl 2> gpurun_out/r4_one.err || { tail -5 gpurun_out/r4_one.err; return 1; }
  python - "$label" <<'PY'
import json, sys
r = json.loads(open('gpurun_out/r4_one.jsonl').read().strip().splitlines()[-1])
r['label'] = sys.argv[1]
open('gpurun_out/r4_ab3.jsonl', 'a').write(json.dumps(r) + '\n')
print(sys.argv[1], r['value'], r.get('p50_latency_ms'), r.get('p99_latency_ms'), r['device_ms_p50'],
      r['cpu_cores_busy_rank0'], r['cpu_cores_by_stage_rank0'], r['step_rate_spread']['range_pct'],
      r.get('latency_stages_ms'))
PY
}
run r50_pack --model resnet50 --steps 10 --warmup 3 || exit 1
run r50_nopack --model resnet50 --steps 10 --warmup 3 --no-text-pack || exit 1
run lenet_sink2 --model lenet5 --steps 20 --warmup 5 || exit 1
run lenet_sink4 --model lenet5 --steps 20 --warmup 5 --sink-parallelism 4 || exit 1
run lenet_sink4_buf8 --model lenet5 --steps 20 --warmup 5 --sink-parallelism 4 --producer-buffer-mb 8 || exit 1
run lenet_nopack --model lenet5 --steps 20 --warmup 5 --no-text-pack || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_prof50 -o run -- python bench.py --model resnet50 --steps 4 --warmup 2 --latency-load 0 > gpurun_out/r4_prof50.log 2>&1 || exit 1
python tools/prof_summary.py $(find gpurun_out/r4_prof50 -name '*.db' | head -1) --top 16 > gpurun_out/r4_prof50.txt 2>&1
cat gpurun_out/r4_prof50.txt | cut -c1-160
