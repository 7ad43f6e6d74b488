# model numerics on logits (calibration prints with -s) + smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r2_models.log 2>&1; rc=$?
grep -E "err|fp8|fused|gemm|passed|failed|Error" gpurun_out/r2_models.log | head -60
[ $rc -eq 0 ] && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
