# config-5 SLO sweep (p99 record e2e <= 5 ms) with the session's final code (32 MB producer buffer)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python tools/slo_sweep.py --slo-ms 5 --rates 1000000,1200000,1300000,1400000 --dtypes bf16,fp8 > gpurun_out/r2_slo_final.jsonl 2> gpurun_out/r2_slo_final.err || { tail -20 gpurun_out/r2_slo_final.err; exit 1; }
cat gpurun_out/r2_slo_final.jsonl
