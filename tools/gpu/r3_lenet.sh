#!/bin/bash
# GPU box: fused LeNet-5 kernel - model tests, forward bench, kernel trace, config-1 end to end
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lenet_tests.log 2>&1 || { tail -30 gpurun_out/lenet_tests.log; exit 1; }
tail -1 gpurun_out/lenet_tests.log
grep "lenet5" gpurun_out/lenet_tests.log | head -5
timeout -k 10 120 python -u -m pytest tests/test_models_gpu.py -q -s -k lenet5_fused > gpurun_out/lenet_fused_err.log 2>&1; grep "lenet5 fused" gpurun_out/lenet_fused_err.log
timeout -k 10 120 python tools/bench_forward.py --model lenet5 --batches 1,64,256,1024,4096 > gpurun_out/lenet_fwd.log 2>&1 || { tail -20 gpurun_out/lenet_fwd.log; exit 1; }
cat gpurun_out/lenet_fwd.log
rm -rf gpurun_out/prof_lenet
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lenet -o l -- python3 tools/bench_forward.py --model lenet5 --batches 256 --iters 50 > gpurun_out/prof_lenet.log 2>&1 || exit 1
cat $(find gpurun_out/prof_lenet -name "*kernel_stats.csv" | head -1) | cut -c1-160 | head -6
timeout -k 10 240 python bench.py --model lenet5 > gpurun_out/lenet_e2e.log 2>&1 || { tail -20 gpurun_out/lenet_e2e.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/lenet_e2e.log") if l.startswith("{")][-1])
print({k: d.get(k) for k in ("value", "p50_latency_ms", "p99_latency_ms", "latency_stages_ms", "device_ms_p50",
                             "json_mb_per_s_rank0", "cpu_cores_busy_rank0", "step_rate_spread", "timed_s")})
PY
