#!/bin/bash
# GPU box: broker zero-copy (vmsplice/splice, like Kafka's sendfile) vs copying writev, alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for args in "--broker-zero-copy" "" "--broker-zero-copy" "" "--broker-zero-copy" ""; do
  timeout -k 10 200 python bench.py $args > gpurun_out/zc_ab.log 2>&1 || { tail -20 gpurun_out/zc_ab.log; exit 1; }
  python - "$args" <<'PY' >> gpurun_out/zc_ab.jsonl
import json, sys
d = json.loads([l for l in open("gpurun_out/zc_ab.log") if l.startswith("{")][-1])
keep = ("value", "step_rate_spread", "json_mb_per_s_rank0", "cpu_cores_busy_rank0",
        "cpu_cores_by_stage_rank0", "device_ms_p50", "p50_latency_ms", "p99_latency_ms",
        "latency_stages_ms")
print(json.dumps({"args": sys.argv[1] or "copy", **{k: d.get(k) for k in keep}}))
PY
  tail -1 gpurun_out/zc_ab.jsonl
done
