# conv_patch on by default (128-channel tiles): full GPU suite, ResNet-50 A/B (GALE_CONV_PATCH=0/1), per-layer times
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_pytest_gpu_full.log 2>&1 || { tail -30 gpurun_out/r2_pytest_gpu_full.log; exit 1; }
tail -1 gpurun_out/r2_pytest_gpu_full.log
for k in 0 1 0 1; do
  GALE_CONV_PATCH=$k timeout -k 10 120 python tools/bench_forward.py --model resnet50 --batches 64,128,256 --iters 30 > gpurun_out/patch.log 2>&1 || { tail -20 gpurun_out/patch.log; exit 1; }
  grep '^{' gpurun_out/patch.log | sed "s/^{/{\"conv_patch\": $k, /"
done
d=gpurun_out/lab/patch_default
rm -rf $d; mkdir -p $d
timeout -k 10 200 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- \
  python3 tools/bench_forward.py --eager --iters 3 --model resnet50 --batches 256 > $d/log 2>&1 || { tail -5 $d/log; exit 1; }
python3 tools/pmc_table.py --label-model resnet50 --batch 256 --trace $(find $d -name '*kernel_trace.csv' | head -1) > $d/table.txt
grep -E "3x3/1|TOTAL" $d/table.txt | cut -c1-60
