#!/bin/bash
# A/B: the bf16 ResNet-20 forward in its 4-wave form (GALE_R20_WAVES=4: 1 wave per SIMD, 77 KB
# of LDS, room on the CU for the ingest passes and a second forward workgroup) vs the default
# 8-wave form (the whole register file, ~150 KB of LDS with the weight prefetch buffer).
# Forward alone, then config 2 interleaved x3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r6nw
mkdir -p $out
for w in ${FWD_WAVES-8 4}; do
  GALE_R20_WAVES=$w timeout -k 10 120 python tools/bench_forward.py --model resnet20 \
      --batches 64,128,256 --iters 50 > $out/fwd_w$w.log 2>&1 || { tail -5 $out/fwd_w$w.log; exit 1; }
  GALE_R20_WAVES=$w timeout -k 10 120 python tools/bench_forward.py --model resnet20 \
      --batches 256 --iters 50 --streams 2 >> $out/fwd_w$w.log 2>&1 || { tail -5 $out/fwd_w$w.log; exit 1; }
  grep '^{' $out/fwd_w$w.log | python -c "import json,sys; [print('w$w', d['batch'], d['streams'], round(d['ms']*1e3,1), 'us') for d in map(json.loads, sys.stdin)]"
done
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
for i in 1 2 3; do
  run w8_$i GALE_R20_WAVES=8 || exit 1
  run w4_$i GALE_R20_WAVES=4 || exit 1
done
