# config-5 latency-SLO sweep at higher offered loads with the current host sizing (bf16 / fp8)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r2_unf_tests.log 2>&1 || { tail -30 gpurun_out/r2_unf_tests.log; exit 1; }
tail -1 gpurun_out/r2_unf_tests.log
grep -h "unfolded-BN rel" gpurun_out/r2_unf_tests.log || true
timeout -k 10 1000 python tools/slo_sweep.py --slo-ms 5 --rates 800000,1000000,1200000,1400000 --dtypes bf16,fp8 > gpurun_out/r2_slo_sweep2.jsonl 2> gpurun_out/r2_slo_sweep2.err || { tail -20 gpurun_out/r2_slo_sweep2.err; exit 1; }
cat gpurun_out/r2_slo_sweep2.jsonl
