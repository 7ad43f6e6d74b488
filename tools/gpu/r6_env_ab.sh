#!/bin/bash
# Runtime-environment A/B on config 2, interleaved: HIP copies on SDMA engines (default) vs blit
# kernels (HSA_ENABLE_SDMA=0), and 4 (HIP's default) vs 8 hardware queues per process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r6e
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
      d["latency_stages_ms"]["ingest"], d.get("latency_ingest_device_us"), flush=True)
PY
}
for i in 1 2; do
  run base_$i GALE_AB=0 || exit 1
  run nosdma_$i HSA_ENABLE_SDMA=0 || exit 1
  run hwq8_$i GPU_MAX_HW_QUEUES=8 || exit 1
done
