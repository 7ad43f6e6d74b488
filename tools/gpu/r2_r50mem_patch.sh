# ResNet-50 b256 per-layer vector-memory path counters (is the conv_gemm k-loop bound by the TA/TD/L2 path?)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
P2="TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES GRBM_GUI_ACTIVE"
d=gpurun_out/pmc_r50mem_patch
rm -rf $d; mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace -d $d/trace -o run --output-format csv -- \
  python3 tools/bench_forward.py --eager --iters 3 --model resnet50 --batches 256 > $d/trace.log 2>&1 || { tail -5 $d/trace.log; exit 1; }
i=1
for P in "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --pmc $P -d $d/p$i -o run --output-format csv -- \
    python3 tools/bench_forward.py --eager --iters 3 --model resnet50 --batches 256 > $d/p$i.log 2>&1 || { tail -5 $d/p$i.log; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_table.py --label-model resnet50 --batch 256 --trace $(find $d/trace -name '*kernel_trace.csv' | head -1) \
  --pmc $(find $d/p1 $d/p2 -name '*counter_collection.csv') \
  --show SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_VMEM,SQ_INST_LEVEL_VMEM,SQ_INSTS_VMEM,SQ_BUSY_CYCLES,TA_TA_BUSY,TA_ADDR_STALLED_BY_TC_CYCLES,TD_TD_BUSY,TD_TC_STALL,TCP_TCC_READ_REQ_LATENCY,TCP_TCC_READ_REQ,TCP_PENDING_STALL_CYCLES > gpurun_out/pmc_r50_mem_patch.txt
cat gpurun_out/pmc_r50_mem_patch.txt | cut -c1-60,95-400
