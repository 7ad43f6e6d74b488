#!/bin/bash
# fused ResNet-20 kernel: numerics tests, forward throughput, PMC (LDS conflicts / MFMA busy)
set -o pipefail
mkdir -p gpurun_out/fused
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_models_gpu.py > gpurun_out/fused/test.log 2>&1 || { tail -30 gpurun_out/fused/test.log; exit 1; }
tail -2 gpurun_out/fused/test.log
timeout -k 10 120 python3 tools/bench_forward.py --model resnet20 --batches 256,1024,4096 --iters 100 > gpurun_out/fused/fwd.jsonl 2>&1 || exit 1
timeout -k 10 120 python3 tools/bench_forward.py --model resnet20 --dtype fp8 --batches 256,4096 --iters 100 >> gpurun_out/fused/fwd.jsonl 2>&1 || exit 1
cat gpurun_out/fused/fwd.jsonl
d=gpurun_out/fused/pmc
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
timeout -k 10 120 rocprofv3 --kernel-trace --kernel-include-regex resnet20_fused -d $d/trace -o run --output-format csv -- \
  python3 tools/bench_forward.py --eager --iters 3 --model resnet20 --batches 256,1024 > $d.trace.log 2>&1 || { tail -5 $d.trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-include-regex resnet20_fused -d $d/p1 -o run --output-format csv -- \
  python3 tools/bench_forward.py --eager --iters 3 --model resnet20 --batches 256,1024 > $d.p1.log 2>&1 || { tail -5 $d.p1.log; exit 1; }
python3 tools/pmc_table.py --trace $(find $d/trace -name '*kernel_trace.csv' | head -1) \
  --pmc $(find $d/p1 -name '*counter_collection.csv') > gpurun_out/fused/pmc.txt
cat gpurun_out/fused/pmc.txt
