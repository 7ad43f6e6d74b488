# ResNet-50 b256 per-layer LDS-pipe counters (is the conv_gemm inner loop LDS-bound?)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P4="SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
d=gpurun_out/pmc_r50lds
rm -rf $d; mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace -d $d/trace -o run --output-format csv -- \
  python3 tools/bench_forward.py --eager --iters 3 --model resnet50 --batches 256 > $d/trace.log 2>&1 || { tail -5 $d/trace.log; exit 1; }
i=1
for P in "$P1" "$P4"; do
  timeout -s KILL 120 rocprofv3 --pmc $P -d $d/p$i -o run --output-format csv -- \
    python3 tools/bench_forward.py --eager --iters 3 --model resnet50 --batches 256 > $d/p$i.log 2>&1 || { tail -5 $d/p$i.log; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_table.py --label-model resnet50 --batch 256 --trace $(find $d/trace -name '*kernel_trace.csv' | head -1) \
  --pmc $(find $d/p1 $d/p2 -name '*counter_collection.csv') \
  --show SQ_LDS_IDX_ACTIVE,SQ_LDS_DATA_FIFO_FULL,SQ_LDS_CMD_FIFO_FULL,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_LDS,SQ_INSTS_LDS_LOAD_BANDWIDTH,SQ_WAIT_INST_ANY,SQ_BUSY_CYCLES > gpurun_out/pmc_r50_lds.txt
cat gpurun_out/pmc_r50_lds.txt
