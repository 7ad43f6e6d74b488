#!/bin/bash
# A/B: the ingest lane's completion wait - a first sleep of ~80 % of the lane's expected device
# time, then 5 us polls (default) vs 20 us polls from the start (GALE_INGEST_POLL_PREDICT=0).
# Config 2 and config 1, interleaved.
# (The predictive wait was not kept: GALE_INGEST_POLL_PREDICT no longer exists, both arms now
# run the same code. Results: profiles/r6_ab_ingest_poll.jsonl.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r6w
mkdir -p $out
run() {  # label, model, env...
  local label=$1 model=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --model $model --steps 10 --warmup 3 \
      > $out/$label.log 2>&1 || { tail -5 $out/$label.log; return 1; }
  python - "$out/$label.log" "$label" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[2], d["value"], d["p50_latency_ms"], d["p99_latency_ms"], d.get("latency_cg_cores"),
      {k: v[0] for k, v in d["latency_stages_ms"].items()}, d.get("latency_ingest_us_per_fetch"),
      flush=True)
PY
}
for i in 1 2; do
  run pred_r20_$i resnet20 GALE_AB=1 || exit 1
  run poll_r20_$i resnet20 GALE_INGEST_POLL_PREDICT=0 || exit 1
  run pred_l5_$i lenet5 GALE_AB=1 || exit 1
  run poll_l5_$i lenet5 GALE_INGEST_POLL_PREDICT=0 || exit 1
done
