#!/bin/bash
# Config 1 (LeNet-5): the GPU-ingest lanes' completion poll interval, 20 us (default) vs 10 vs 40
# (GALE_INGEST_POLL_US), interleaved x3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r6pl
mkdir -p $out
for i in 1 2 3; do
  for p in 20 40; do
    GALE_INGEST_POLL_US=$p timeout -k 10 200 python bench.py --model lenet5 --steps 10 --warmup 3 > $out/p${p}_$i.log 2>&1 || exit 1
    python - "$out/p${p}_$i.log" "p${p}_$i" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[2], d["value"], d["p50_latency_ms"], d["p99_latency_ms"], d.get("latency_cg_cores"),
      d["latency_stages_ms"]["ingest"][:2], d["latency_ingest_us_per_fetch"]["device_wait"],
      d["cpu_cores_by_stage_rank0"]["decode"], flush=True)
PY
  done
done
