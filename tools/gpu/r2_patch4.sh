# conv_patch 64-channel single-patch tiles at 4 WG per CU (GALE_CONV_PATCH_OCC=4): tests, ResNet-50 A/B, per-layer times
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
GALE_CONV_PATCH_OCC=4 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -k "patch or (resnet50 and not fp8)" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/patch3_test.log 2>&1 || { tail -40 gpurun_out/patch3_test.log; exit 1; }
tail -1 gpurun_out/patch3_test.log
for k in 2 4 2 4; do
  GALE_CONV_PATCH_OCC=$k timeout -k 10 120 python tools/bench_forward.py --model resnet50 --batches 64,256 --iters 30 > gpurun_out/patch3.log 2>&1 || { tail -20 gpurun_out/patch3.log; exit 1; }
  grep '^{' gpurun_out/patch3.log | sed "s/^{/{\"patch_occ\": $k, /" | cut -c1-150
done
d=gpurun_out/lab/patch_occ4
rm -rf $d; mkdir -p $d
GALE_CONV_PATCH_OCC=4 timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- \
  python3 tools/bench_forward.py --eager --iters 3 --model resnet50 --batches 256 > $d/log 2>&1 || { tail -5 $d/log; exit 1; }
python3 tools/pmc_table.py --label-model resnet50 --batch 256 --trace $(find $d -name '*kernel_trace.csv' | head -1) > $d/table.txt
grep -E "3x3/1|TOTAL" $d/table.txt | cut -c1-60
