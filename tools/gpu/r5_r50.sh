#!/bin/bash
# ResNet-50 with the fused 56x56 bottlenecks: kernel A/B, forward A/B (1 and 2 streams),
# per-layer kernel trace + PMC table, config 4 end to end x3.
set -o pipefail
d=gpurun_out/r50
mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 120 python tools/bench_bneck.py --layered > $d/kern.jsonl 2> $d/err.log || { tail $d/err.log; exit 1; }
cat $d/kern.jsonl
: > $d/fwd_ab.jsonl
for r in 1 2; do
  for f in "--no-fuse-blocks" "" "--no-fuse-blocks --streams 2" "--streams 2"; do
    timeout -k 10 200 python tools/bench_forward.py --model resnet50 --batches 256 --iters 30 $f \
        >> $d/fwd_ab.jsonl 2>> $d/err.log || { tail -20 $d/err.log; exit 1; }
  done
done
cat $d/fwd_ab.jsonl
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
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 > $d/c4_$i.json 2> $d/c4_$i.err \
      || { tail -5 $d/c4_$i.err; exit 1; }
  tail -1 $d/c4_$i.json | cut -c1-300
done
