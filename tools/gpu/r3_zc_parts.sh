#!/bin/bash
# GPU box: input partitions (= source threads) per GPU with the zero-copy broker, alternating;
# then a world-2 shared-GPU rehearsal with the zero-copy default
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for args in "--partitions 12" "--partitions 16" "--partitions 24" "--partitions 12" "--partitions 16" "--partitions 24"; do
  timeout -k 10 200 python bench.py --latency-load 0 $args > gpurun_out/zcp.log 2>&1 || { tail -20 gpurun_out/zcp.log; exit 1; }
  python - "$args" <<'PY' >> gpurun_out/zc_parts.jsonl
import json, sys
d = json.loads([l for l in open("gpurun_out/zcp.log") if l.startswith("{")][-1])
keep = ("value", "step_rate_spread", "json_mb_per_s_rank0", "cpu_cores_busy_rank0",
        "cpu_cores_by_stage_rank0")
print(json.dumps({"args": sys.argv[1], **{k: d.get(k) for k in keep}}))
PY
  tail -1 gpurun_out/zc_parts.jsonl | cut -c1-300
done
timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 1 --shared-gpu-rehearsal \
  --steps 10 --warmup 3 > gpurun_out/rehearsal_w2.log 2>&1 || { tail -30 gpurun_out/rehearsal_w2.log; exit 1; }
grep '^{' gpurun_out/rehearsal_w2.log | tail -1 | cut -c1-300
