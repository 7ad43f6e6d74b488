#!/bin/bash
# The ingest plan carried by the text's DMA (one H2D per fetch instead of two): engine GPU tests,
# then config 2 and config 1 with sampled device timing (latency_ingest_device_us).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r6p
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 \
    --timeout-method thread > $out/pytest_engine.log 2>&1 || { tail -30 $out/pytest_engine.log; exit 1; }
tail -1 $out/pytest_engine.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $out/c2_$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --model lenet5 --steps 10 --warmup 3 > $out/c1_$i.log 2>&1 || exit 1
done
python - <<'PY'
import json
for f in ["c2_1", "c1_1", "c2_2", "c1_2"]:
    l = [x for x in open(f"gpurun_out/r6p/{f}.log") if x.startswith("{")][-1]
    d = json.loads(l)
    print(f, d["value"], d["p50_latency_ms"], d["p99_latency_ms"],
          d["latency_stages_ms"]["ingest"], d.get("latency_ingest_device_us"))
PY
