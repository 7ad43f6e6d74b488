#!/bin/bash
# Config 2 steady state on the final code: 100-step windows x2 and one 300-step soak, then the
# kernel trace of the default bench (PART=c of r6_final.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r6soak
mkdir -p $out
for r in s100_1:100 s100_2:100 s300:300; do
  label=${r%%:*}; steps=${r##*:}
  timeout -k 10 400 python -u bench.py --steps $steps --warmup 5 > $out/$label.log 2>&1 || { tail -5 $out/$label.log; exit 1; }
  python - "$out/$label.log" "$label" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
r = d["step_rates"]
w = [sum(r[i:i + 30]) / len(r[i:i + 30]) for i in range(0, len(r), 30)]
print(sys.argv[2], d["value"], d["p50_latency_ms"], d["p99_latency_ms"], d["p999_latency_ms"],
      d["timed_s"], "30-step windows", [round(x / 1e6, 3) for x in w], flush=True)
PY
done
PART=c bash tools/gpu/r6_final.sh
