# conv_patch two-image 7x7 tiles: kernel + model tests, per-layer times (GALE_CONV_PATCH_MULTI=1 default vs 0), forward A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -k "patch or resnet50" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/p7_test.log 2>&1 || { tail -40 gpurun_out/p7_test.log; exit 1; }
tail -1 gpurun_out/p7_test.log
for v in 1 0; do
  d=gpurun_out/lab/multi$v
  rm -rf $d; mkdir -p $d
  GALE_CONV_PATCH_MULTI=$v timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- \
    python3 tools/bench_forward.py --eager --iters 3 --model resnet50 --batches 256 > $d/log 2>&1 || { tail -5 $d/log; exit 1; }
  python3 tools/pmc_table.py --label-model resnet50 --batch 256 --trace $(find $d -name '*kernel_trace.csv' | head -1) > $d/table.txt
  echo "== MULTI=$v"; grep -E "3x3/1 512|TOTAL" $d/table.txt | cut -c1-60
done
for v in 1 0 1 0; do
  GALE_CONV_PATCH_MULTI=$v timeout -k 10 120 python tools/bench_forward.py --model resnet50 --batches 64,256 --iters 30 > gpurun_out/p7.log 2>&1 || { tail -20 gpurun_out/p7.log; exit 1; }
  grep '^{' gpurun_out/p7.log | sed "s/^{/{\"multi\": $v, /" | cut -c1-150
done
