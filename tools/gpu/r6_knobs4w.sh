#!/bin/bash
# Host-pipeline sizing re-check on the final code (config 2), interleaved x2: the defaults
# (6 replicas, 10 ingest lanes) against one change each, with the 4-wave forward.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r6k3
mkdir -p $out
run() {  # label, bench args...
  local label=$1; shift
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 "$@" > $out/$label.log 2>&1 || {
    tail -5 $out/$label.log; return 1; }
  python - "$out/$label.log" "$label" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[2], d["value"], d["p50_latency_ms"], d["p99_latency_ms"], d["cpu_cores_busy_rank0"],
      d["step_rate_spread"]["range_pct"], flush=True)
PY
}
for i in 1 2; do
  run base_$i || exit 1
  run d12_$i --decode-threads 12 || exit 1
  run r8_$i --replicas-per-gpu 8 || exit 1
  run r4_$i --replicas-per-gpu 4 || exit 1
  run d8_$i --decode-threads 8 || exit 1
done
