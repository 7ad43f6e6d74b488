#!/bin/bash
# GPU-box: GPU tests, then bench.py on the BASELINE.json configurations (1 GPU):
#   config 1 (LeNet-5, MNIST 28x28x1 plumbing), config 2 (headline: ResNet-20 bf16), config 4 (ResNet-50 bf16, batch <= 256, 224x224x3
#   records), config 5 (ResNet-20 fp8, latency-SLO mode: small batches, short max-wait).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/cfg_$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 gpurun_out/cfg_$name.log
  return $rc
}
run c1_lenet5_bf16 --model lenet5 --steps 100 --warmup 10 || exit $?
run c2_resnet20_bf16 --steps 100 --warmup 10 || exit $?
run c4_resnet50_bf16 --model resnet50 --batch 64 --replicas-per-gpu 2 --partitions 4 --source-parallelism 4 --decode-threads 4 --steps 30 --warmup 5 --distinct 64 || exit $?
run c5_resnet20_fp8_slo --dtype fp8 --batch 32 --max-wait-us 200 --steps 200 --warmup 20 || exit $?
# latency at a fixed offered load (open-loop feeder), fp8 and bf16
for r in ${RATES:-100000 300000}; do
  run c5_fp8_rate$r --dtype fp8 --batch 32 --max-wait-us 200 --rate $r --steps 400 --warmup 40 || exit $?
  run c2_bf16_rate$r --batch 32 --max-wait-us 200 --rate $r --steps 400 --warmup 40 || exit $?
done
