#!/bin/bash
# The latency phase's producer batch size on config 2, interleaved: 64 records per batch (the
# backlog's batches, the default) vs 32 and 16 (closer to a kafka-clients producer, whose 16 KB
# batch.size sends one ~35 KB record per batch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r6l
mkdir -p $out
for i in 1 2; do
  for b in 64 32 16; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --latency-batch-records $b \
        > $out/b${b}_$i.log 2>&1 || exit 1
    python - "$out/b${b}_$i.log" "b${b}_$i" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[2], d["value"], d["p50_latency_ms"], d["p99_latency_ms"], d["p999_latency_ms"],
      d.get("latency_cg_cores"), {k: v[0] for k, v in d["latency_stages_ms"].items()}, flush=True)
PY
  done
done
