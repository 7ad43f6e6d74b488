# PMC evidence for the conv / fused kernels: one rocprofv3 pass per counter group (each within
# the per-block limits), eager launches (per-dispatch attribution), plus a kernel-trace pass
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="FETCH_SIZE"
P3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
run_case() {  # name, regex, bench args
  local name=$1 rx=$2; shift 2
  local d=gpurun_out/pmc_$name
  rm -rf $d; mkdir -p $d
  timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "$rx" -d $d/trace -o run --output-format csv -- \
    python3 tools/bench_forward.py --eager --iters 3 "$@" > $d/trace.log 2>&1 || { echo "trace $name failed"; tail -5 $d/trace.log; return 1; }
  local i=1
  for P in "$P1" "$P2" "$P3"; do
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$rx" -d $d/p$i -o run --output-format csv -- \
      python3 tools/bench_forward.py --eager --iters 3 "$@" > $d/p$i.log 2>&1 || { echo "pmc $name pass $i failed"; tail -5 $d/p$i.log; return 1; }
    i=$((i+1))
  done
  python3 tools/pmc_table.py --trace $(find $d/trace -name '*kernel_trace.csv' | head -1) \
    --pmc $(find $d/p1 $d/p2 $d/p3 -name '*counter_collection.csv') > gpurun_out/pmc_$name.txt
  head -30 gpurun_out/pmc_$name.txt
}
run_case r50b256 'conv_gemm|conv_mfma' --model resnet50 --batches 256 && \
run_case r20 'resnet20_fused' --model resnet20 --batches 256,1024
