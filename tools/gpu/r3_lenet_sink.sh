#!/bin/bash
# GPU box: config 1 (LeNet-5) end to end A/B over sink settings (default: producer buffer 32 vs 8 MB)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for args in ${LENET_ARGS:-"--producer-buffer-mb 32" "--producer-buffer-mb 8"}; do
  timeout -k 10 240 python bench.py --model lenet5 $args > gpurun_out/lenet_sink.log 2>&1 || { tail -20 gpurun_out/lenet_sink.log; exit 1; }
  python3 - "$args" <<'PY' | tee -a gpurun_out/lenet_sink.jsonl
import json, sys
d = json.loads([l for l in open("gpurun_out/lenet_sink.log") if l.startswith("{")][-1])
print(json.dumps({"args": sys.argv[1], **{k: d.get(k) for k in ("value", "p50_latency_ms", "p99_latency_ms",
      "latency_stages_ms", "device_ms_p50", "cpu_cores_busy_rank0", "cpu_cores_by_stage_rank0", "step_rate_spread")}}))
PY
done
