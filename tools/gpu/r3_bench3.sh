#!/bin/bash
# GPU box: three default bench.py runs back to back (the driver's N = 1 command)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
rm -f gpurun_out/b3.jsonl
for i in 1 2 3; do
  timeout -k 10 240 python bench.py "$@" > gpurun_out/b3.log 2>&1 || { tail -20 gpurun_out/b3.log; exit 1; }
  grep '^{' gpurun_out/b3.log | tail -1 >> gpurun_out/b3.jsonl
  python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/b3.jsonl").read().splitlines()[-1])
print(d["value"], d["timed_s"], d["step_rate_spread"], d["p50_latency_ms"], d["p99_latency_ms"],
      d["cpu_cores_busy_rank0"])
PY
done
