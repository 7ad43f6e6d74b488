#!/bin/bash
# GPU box: full GPU suite (one process), three default bench runs, a rocprofv3 kernel trace of
# the default serving configuration. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/bench_3runs.jsonl
for i in 1 2 3; do
  timeout -k 10 240 python bench.py > gpurun_out/bench_run.log 2>&1 || { tail -20 gpurun_out/bench_run.log; exit 1; }
  grep '^{' gpurun_out/bench_run.log | tail -1 >> gpurun_out/bench_3runs.jsonl
  python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_3runs.jsonl").read().splitlines()[-1])
print({k: d.get(k) for k in ("value", "p50_latency_ms", "p99_latency_ms", "cpu_cores_busy_rank0")},
      d["step_rate_spread"]["range_pct"], d["cpu_cores_by_stage_rank0"])
PY
done
bash tools/gpu/r3_prof.sh
