#!/bin/bash
# GPU box: latency phases at 0.5/0.7/0.9 x max (2 repeats) with zero-copy and copying brokers,
# per-phase TCP counters (retransmits, RTOs, receive pruning, zero windows) next to the p99
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for args in "--broker-zero-copy" "--no-broker-zero-copy"; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --latency-sweep 0.5,0.7,0.9 --latency-repeat 2 $args > gpurun_out/tail_tcp.log 2>&1 || { tail -20 gpurun_out/tail_tcp.log; exit 1; }
  python - "$args" <<'PY' | tee -a gpurun_out/tail_tcp.txt
import json, sys
d = json.loads([l for l in open("gpurun_out/tail_tcp.log") if l.startswith("{")][-1])
print(sys.argv[1], "value", d["value"], "p50/p99", d["p50_latency_ms"], d["p99_latency_ms"], "tcp", d.get("latency_tcp"))
for x in d.get("latency_sweep", []):
    print(" ", x["load"], "p50", x["p50_ms"], "p99", x["p99_ms"], "bs_p99", x["stages_ms"]["broker_source"][1], "tcp", x.get("tcp"))
PY
done
