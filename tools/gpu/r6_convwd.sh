#!/bin/bash
# conv_gemm with its weight fragments loaded straight from global memory (GALE_CONV_WD=1: only
# the im2col rows go through LDS-DMA) vs LDS-staged weights (default): single layers at batch
# 256 / 128 (tools/bench_conv.py), the ResNet-50 forward, and the model numerics under WD.
# (The weights-direct form was not kept: GALE_CONV_WD no longer exists, both arms now run the
# same code. Results: profiles/r6_conv_wdirect_ab.jsonl.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r6wd
mkdir -p $out
GALE_CONV_WD=1 timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py \
    -q -k "resnet50 or conv" --timeout 240 --timeout-method thread > $out/pytest_wd.log 2>&1 \
    || { tail -30 $out/pytest_wd.log; exit 1; }
tail -1 $out/pytest_wd.log
for i in 1 2; do
  for w in 0 1; do
    for b in 256 128; do
      GALE_CONV_WD=$w timeout -k 10 120 python tools/bench_conv.py --batch $b --tag wd${w}_b${b}_$i \
          >> $out/conv.jsonl 2> $out/conv.err || { tail -5 $out/conv.err; exit 1; }
    done
    GALE_CONV_WD=$w timeout -k 10 180 python tools/bench_forward.py --model resnet50 \
        --batches 128,256 --iters 20 > $out/fwd_wd${w}_$i.log 2>&1 || { tail -5 $out/fwd_wd${w}_$i.log; exit 1; }
    grep '^{' $out/fwd_wd${w}_$i.log | python -c "import json,sys; [print('wd$w', json.loads(l)['batch'], round(json.loads(l)['ms'],3)) for l in sys.stdin]"
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r6wd/conv.jsonl"):
    d = json.loads(l); print(d["tag"], d["layer"], d["us"], d["tflops"], "%.1e" % d["rel_err"])
PY
