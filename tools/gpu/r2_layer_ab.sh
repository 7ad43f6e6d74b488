# ResNet-50 b256 per-layer kernel times under each conv_gemm variant switch (kernel trace only)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "X=0" "GALE_GEMM_BM256=2" "GALE_GEMM_BM256=1" "GALE_GEMM_BM256=5" "GALE_GEMM_RS=1" "GALE_GEMM_RING=1" "GALE_GEMM_BM256=3"; do
  d=gpurun_out/lab/${v//=/_}
  rm -rf $d; mkdir -p $d
  env $v true
  export $v
  timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- \
    python3 tools/bench_forward.py --eager --iters 3 --model resnet50 --batches 256 > $d/log 2>&1 || { tail -5 $d/log; exit 1; }
  unset ${v%%=*}
  python3 tools/pmc_table.py --label-model resnet50 --batch 256 --trace $(find $d -name '*kernel_trace.csv' | head -1) > $d/table.txt
  echo "$v $(tail -1 $d/table.txt)"
done
