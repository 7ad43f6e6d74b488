#!/bin/bash
# A/B: replica streams kept off the last N CUs (GALE_REPLICA_CU_RESERVE) so the GPU ingest's
# passes do not queue behind whole-chip forward batches. Config 2, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r6c
mkdir -p $out
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $out/$label.log 2>&1 || {
    tail -5 $out/$label.log; return 1; }
  python - "$out/$label.log" "$label" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[2], d["value"], d["p50_latency_ms"], d["p99_latency_ms"], d["device_ms_p50"],
      {k: v[0] for k, v in d["latency_stages_ms"].items()}, d.get("latency_ingest_device_us"),
      flush=True)
PY
}
for i in 1 2; do
  run base_$i GALE_AB=0 || exit 1
  run res32_$i GALE_REPLICA_CU_RESERVE=32 || exit 1
  run res16_$i GALE_REPLICA_CU_RESERVE=16 || exit 1
done
