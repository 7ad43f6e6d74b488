#!/bin/bash
# Config 2 with the 4-wave forward: 12 ingest lanes (default) vs 14, interleaved x4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r6l14
mkdir -p $out
for i in 1 2 3 4; do
  for d in 12 14; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --decode-threads $d > $out/d${d}_$i.log 2>&1 || exit 1
    python - "$out/d${d}_$i.log" "d${d}_$i" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[2], d["value"], d["p50_latency_ms"], d["p99_latency_ms"], d["cpu_cores_busy_rank0"],
      d["step_rate_spread"]["range_pct"], flush=True)
PY
  done
done
