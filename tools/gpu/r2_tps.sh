# barrier cadence A/B in conv_patch: 64-channel tiles with 1 vs 2 taps per k-step (GALE_CONV_PATCH_TPS=1/2), default for reference
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
GALE_CONV_PATCH_TPS=2 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -k "(patch and not case0 and not 56-64) or (resnet50 and not fp8)" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tps_test.log 2>&1 || { tail -40 gpurun_out/tps_test.log; exit 1; }
tail -1 gpurun_out/tps_test.log
for v in 0 1 2; do
  d=gpurun_out/lab/tps$v
  rm -rf $d; mkdir -p $d
  GALE_CONV_PATCH_TPS=$v timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- \
    python3 tools/bench_forward.py --eager --iters 3 --model resnet50 --batches 256 > $d/log 2>&1 || { tail -5 $d/log; exit 1; }
  python3 tools/pmc_table.py --label-model resnet50 --batch 256 --trace $(find $d -name '*kernel_trace.csv' | head -1) > $d/table.txt
  echo "== TPS=$v"; grep -E "3x3/1 (128|256)|TOTAL" $d/table.txt | cut -c1-60
done
