# config-5 SLO sweep with the final controller and producer defaults
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python tools/slo_sweep.py --slo-ms 5 --rates 1000000,1100000,1200000,1300000 --dtypes fp8,bf16 > gpurun_out/r2_slo_final2.jsonl 2> gpurun_out/r2_slo_final2.err || { tail -20 gpurun_out/r2_slo_final2.err; exit 1; }
cat gpurun_out/r2_slo_final2.jsonl
