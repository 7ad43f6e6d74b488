# config-5 SLO sweep after the controller's backlog fix
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python tools/slo_sweep.py --slo-ms 5 --rates 1000000,1200000,1300000 --dtypes bf16,fp8 > gpurun_out/r2_slo_sweep3.jsonl 2> gpurun_out/r2_slo_sweep3.err || { tail -20 gpurun_out/r2_slo_sweep3.err; exit 1; }
cat gpurun_out/r2_slo_sweep3.jsonl
