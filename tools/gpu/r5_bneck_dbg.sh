#!/bin/bash
# Phase costs of the fused bottleneck (GALE_BNECK_DBG skip bits) and its PMC counters.
set -o pipefail
d=gpurun_out/bneck_dbg
mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 120 python tools/bench_bneck.py --layered > $d/dbg.jsonl 2> $d/err.log || { tail $d/err.log; exit 1; }
for b in ${DBG:-1 2 4 16 7 23}; do
  GALE_BNECK_DBG=$b timeout -k 10 120 python tools/bench_bneck.py >> $d/dbg.jsonl 2>> $d/err.log || { tail $d/err.log; exit 1; }
done
cat $d/dbg.jsonl
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES"
P2="FETCH_SIZE TA_TA_BUSY_sum TD_TD_BUSY_sum"
P3="WRITE_SIZE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM"
[ -n "$PMC" ] || exit 0
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $d/pmc$i -o run --output-format csv -- \
      python tools/bench_bneck.py --iters 3 > $d/pmc$i.log 2>&1 || { tail -5 $d/pmc$i.log; exit 1; }
  f=$(find $d/pmc$i -name '*counter_collection.csv' | head -1)
  [ -n "$f" ] && cp $f $d/pmc$i.csv
  rm -rf $d/pmc$i
done
ls $d
