#!/bin/bash
# json_parse A/B (gale/_ab/_C.so = the variant) and PMC of the parse-only kernel.
set -o pipefail
d=gpurun_out/json
mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 120 python tools/bench_json.py --batches 256,1024 > $d/base.jsonl 2>&1 || { tail $d/base.jsonl; exit 1; }
cat $d/base.jsonl | grep kernel
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM \
    --output-format csv -d $d/p1 -o run -- python tools/bench_json.py --batches 256 --iters 3 > $d/p1.log 2>&1 || { tail -5 $d/p1.log; exit 1; }
cp $(find $d/p1 -name '*counter_collection.csv' | head -1) $d/pmc1.csv; rm -rf $d/p1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d $d/p2 -o run -- python tools/bench_json.py --batches 256 --iters 3 > $d/p2.log 2>&1 || { tail -5 $d/p2.log; exit 1; }
cp $(find $d/p2 -name '*counter_collection.csv' | head -1) $d/pmc2.csv; rm -rf $d/p2
if [ -f gale/_ab/_C.so ]; then
  cp gale/_C.so $d/_C_base.so.keep 2>/dev/null; cp gale/_ab/_C.so gale/_C.so
  timeout -k 10 120 python tools/bench_json.py --batches 256,1024 > $d/variant.jsonl 2>&1 || { tail $d/variant.jsonl; exit 1; }
  cat $d/variant.jsonl | grep kernel
fi
rm -f $d/_C_base.so.keep
