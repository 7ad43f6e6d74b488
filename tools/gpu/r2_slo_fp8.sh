# config-5 fp8 repeat: is the 1.0 M p99 outlier systematic?
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 600 python tools/slo_sweep.py --slo-ms 5 --rates 1000000,1100000,1200000 --dtypes fp8 > gpurun_out/r2_slo_fp8_$i.jsonl 2> gpurun_out/r2_slo_fp8.err || { tail -20 gpurun_out/r2_slo_fp8.err; exit 1; }
cat gpurun_out/r2_slo_fp8_$i.jsonl
done
