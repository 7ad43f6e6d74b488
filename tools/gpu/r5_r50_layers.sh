#!/bin/bash
# ResNet-50 per-layer table with the final plan (fused stem + pool, 56x56 blocks, projections in
# conv3): kernel trace + three PMC passes -> tools/pmc_table.py.
set -o pipefail
d=gpurun_out/r50b
mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $d/tr -o run -- \
    python tools/bench_forward.py --model resnet50 --batches 256 --iters 5 --eager > $d/tr.log 2>&1 \
    || { tail $d/tr.log; exit 1; }
cp $(find $d/tr -name '*kernel_trace.csv' | head -1) $d/trace.csv
rm -rf $d/tr
i=0
for P in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16" \
         "FETCH_SIZE GRBM_GUI_ACTIVE TD_TD_BUSY_sum TA_TA_BUSY_sum" \
         "WRITE_SIZE GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $d/pmc$i -o run -- \
      python tools/bench_forward.py --model resnet50 --batches 256 --iters 2 --eager \
      > $d/pmc$i.log 2>&1 || { tail -5 $d/pmc$i.log; exit 1; }
  cp $(find $d/pmc$i -name '*counter_collection.csv' | head -1) $d/pmc$i.csv
  rm -rf $d/pmc$i
done
python tools/pmc_table.py --trace $d/trace.csv --pmc $d/pmc1.csv $d/pmc2.csv $d/pmc3.csv \
    --label-model resnet50 --batch 256 --show TD_TD_BUSY_sum,TA_TA_BUSY_sum > $d/layers.txt 2>&1
tail -5 $d/layers.txt
