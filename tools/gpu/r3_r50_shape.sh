#!/bin/bash
# GPU box: config-4 (ResNet-50) host pipeline shape A/B (decode lanes, replicas per GPU), backlog only
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for args in "" "--decode-threads 8" "--replicas-per-gpu 3" "--decode-threads 8 --replicas-per-gpu 3" "--partitions 16 --decode-threads 8"; do
  timeout -k 10 200 python bench.py --model resnet50 --steps 10 --warmup 3 --latency-load 0 $args > gpurun_out/r50_ab.log 2>&1 || { tail -20 gpurun_out/r50_ab.log; exit 1; }
  python - "$args" <<'PY' >> gpurun_out/r50_ab.jsonl
import json, sys
d = json.loads([l for l in open("gpurun_out/r50_ab.log") if l.startswith("{")][-1])
keep = ("value", "step_rate_spread", "json_mb_per_s_rank0", "cpu_cores_busy_rank0",
        "cpu_cores_by_stage_rank0", "device_ms_p50", "batch_images_mean", "backlog_fetch_to_ack_ms_p50")
print(json.dumps({"args": sys.argv[1], **{k: d.get(k) for k in keep}}))
PY
  tail -1 gpurun_out/r50_ab.jsonl
done
