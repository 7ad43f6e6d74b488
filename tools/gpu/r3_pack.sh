#!/bin/bash
# GPU box: nibble transport A/B (pack micro-bench, device unpack tests, bench with/without packing)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python tools/bench_pack.py > gpurun_out/pack_micro.jsonl 2>&1 || exit $?
cat gpurun_out/pack_micro.jsonl
timeout -k 10 300 python -u -m pytest tests/test_text_pack.py -x -q --timeout 60 --timeout-method thread > gpurun_out/pack_tests.log 2>&1 || { tail -20 gpurun_out/pack_tests.log; exit 1; }
tail -1 gpurun_out/pack_tests.log
for cfg in "GALE_TAP_CHUNK_KB=256 GALE_TAP_NOPACK=1" "GALE_TAP_CHUNK_KB=1024" "GALE_TAP_CHUNK_KB=4096" "GALE_TAP_CHUNK_KB=1024 GALE_TAP_NOPACK=1" "GALE_TAP_CHUNK_KB=65536 GALE_TAP_NOPACK=1"; do
  env $cfg timeout -k 10 200 python bench.py --latency-load 0 > gpurun_out/pack_ab.log 2>&1 || { tail -20 gpurun_out/pack_ab.log; exit 1; }
  python - "$cfg" <<'PY' >> gpurun_out/pack_ab.jsonl
import json, sys
d = json.loads([l for l in open("gpurun_out/pack_ab.log") if l.startswith("{")][-1])
keep = ("value", "step_rate_spread", "json_mb_per_s_rank0", "link_ratio_rank0", "cpu_cores_busy_rank0",
        "cpu_cores_by_stage_rank0", "device_ms_p50", "backlog_fetch_to_ack_ms_p50")
print(json.dumps({"args": sys.argv[1], **{k: d.get(k) for k in keep}}))
PY
  tail -1 gpurun_out/pack_ab.jsonl
done
