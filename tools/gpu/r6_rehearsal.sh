#!/bin/bash
# Multi-rank rehearsal on the one-GPU box through the driver's entry point: bench.py --gpus N
# --shared-gpu-rehearsal (N ranks on GPU 0, gloo group), N = 2 and 4.
set -o pipefail
d=gpurun_out/reh
mkdir -p $d
for n in ${NS:-2 4}; do
  timeout -k 10 400 python bench.py --gpus $n --shared-gpu-rehearsal --steps 10 --warmup 3 \
      > $d/w$n.json 2> $d/w$n.err || { echo "FAIL $n"; tail -20 $d/w$n.err; exit 1; }
  python - $d/w$n.json <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(r["n_gpus"], r["value"], r["config"]["parallelism"], "p50", r.get("p50_latency_ms"),
      "p99", r.get("p99_latency_ms"),
      [(x.get("rank"), x.get("images"), x.get("partitions")) for x in r.get("ranks", [])])
PY
done
