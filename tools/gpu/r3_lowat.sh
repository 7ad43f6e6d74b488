#!/bin/bash
# GPU box: consumer receive low-water mark A/B (0 = wake per segment vs 1 MiB), alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for args in "--recv-lowat-kb 0" "--recv-lowat-kb 1024" "--recv-lowat-kb 0" "--recv-lowat-kb 1024" "--recv-lowat-kb 256"; do
  timeout -k 10 200 python bench.py $args > gpurun_out/lowat.log 2>&1 || { tail -20 gpurun_out/lowat.log; exit 1; }
  python3 - "$args" <<'PY' | tee -a gpurun_out/lowat.jsonl
import json, sys
d = json.loads([l for l in open("gpurun_out/lowat.log") if l.startswith("{")][-1])
print(json.dumps({"args": sys.argv[1], **{k: d.get(k) for k in ("value", "p50_latency_ms", "p99_latency_ms",
      "cpu_cores_busy_rank0", "cpu_cores_by_stage_rank0", "step_rate_spread", "json_mb_per_s_rank0")}}))
PY
done
