#!/bin/bash
# fused ResNet-20 fp8 vs bf16: forward times and PMC (MFMA busy, LDS conflicts) at serving batch
set -o pipefail
mkdir -p gpurun_out/fp8
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_models_gpu.py tests/test_engine_gpu.py > gpurun_out/fp8/test.log 2>&1 || { tail -30 gpurun_out/fp8/test.log; exit 1; }
tail -1 gpurun_out/fp8/test.log
timeout -k 10 120 python3 tools/bench_forward.py --model resnet20 --batches 64,256,1024,4096 --iters 100 > gpurun_out/fp8/fwd.jsonl 2>&1 || exit 1
timeout -k 10 120 python3 tools/bench_forward.py --model resnet20 --dtype fp8 --batches 64,256,1024,4096 --iters 100 >> gpurun_out/fp8/fwd.jsonl 2>&1 || exit 1
grep '^{' gpurun_out/fp8/fwd.jsonl | cut -c1-160
d=gpurun_out/fp8/pmc
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_FP8 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
timeout -k 10 120 rocprofv3 --kernel-trace --kernel-include-regex resnet20_fused -d $d/trace -o run --output-format csv -- \
  python3 tools/bench_forward.py --eager --iters 3 --model resnet20 --dtype fp8 --batches 256,1024 > $d.trace.log 2>&1 || { tail -5 $d.trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-include-regex resnet20_fused -d $d/p1 -o run --output-format csv -- \
  python3 tools/bench_forward.py --eager --iters 3 --model resnet20 --dtype fp8 --batches 256,1024 > $d.p1.log 2>&1 || { tail -5 $d.p1.log; exit 1; }
python3 tools/pmc_table.py --mops SQ_INSTS_VALU_MFMA_MOPS_FP8 --trace $(find $d/trace -name '*kernel_trace.csv' | head -1) \
  --pmc $(find $d/p1 -name '*counter_collection.csv') > gpurun_out/fp8/pmc.txt 2>&1
head -8 gpurun_out/fp8/pmc.txt
