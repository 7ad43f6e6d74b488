#!/bin/bash
# Config 2 with the 4-wave forward: max_batch 256 (default) vs 128, interleaved x3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r6b4
mkdir -p $out
for i in 1 2 3; do
  for b in 256 128; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --batch $b > $out/b${b}_$i.log 2>&1 || exit 1
    python - "$out/b${b}_$i.log" "b${b}_$i" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[2], d["value"], d["p50_latency_ms"], d["p99_latency_ms"], d["device_ms_p50"],
      {k: v[0] for k, v in d["latency_stages_ms"].items()}, flush=True)
PY
  done
done
