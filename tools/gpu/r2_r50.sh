# ResNet-50 forward: tests, A/B timing (single-stage K=64 GEMM form), per-layer PMC/roofline table
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_r50_tests.log 2>&1 || { tail -30 gpurun_out/r2_r50_tests.log; exit 1; }
tail -1 gpurun_out/r2_r50_tests.log
for ss in 0 1; do
  GALE_GEMM_SINGLE_STAGE=$ss timeout -k 10 240 python tools/bench_forward.py --model resnet50 --batches 64,128,256 --iters 20 > gpurun_out/r2_r50_ss$ss.log 2>&1 || { tail -20 gpurun_out/r2_r50_ss$ss.log; exit 1; }
  sed "s/^{/{\"single_stage\": $ss, /" gpurun_out/r2_r50_ss$ss.log | grep '^{'
done
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="FETCH_SIZE"
P3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
d=gpurun_out/pmc_r50L
rm -rf $d; mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace -d $d/trace -o run --output-format csv -- \
  python3 tools/bench_forward.py --eager --iters 3 --model resnet50 --batches 256 > $d/trace.log 2>&1 || { tail -5 $d/trace.log; exit 1; }
i=1
for P in "$P1" "$P2" "$P3"; do
  timeout -s KILL 120 rocprofv3 --pmc $P -d $d/p$i -o run --output-format csv -- \
    python3 tools/bench_forward.py --eager --iters 3 --model resnet50 --batches 256 > $d/p$i.log 2>&1 || { tail -5 $d/p$i.log; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_table.py --label-model resnet50 --batch 256 --trace $(find $d/trace -name '*kernel_trace.csv' | head -1) \
  --pmc $(find $d/p1 $d/p2 $d/p3 -name '*counter_collection.csv') > gpurun_out/pmc_r50_layers.txt
cat gpurun_out/pmc_r50_layers.txt
