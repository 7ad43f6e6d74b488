#!/bin/bash
# GPU-box: rocprofv3 kernel traces of the forward-only benchmark, one run per (dtype, batch).
# usage: PROF_CASES="bf16:256 fp8:256" bash tools/gpu_prof_fwd.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MODEL=${MODEL:-resnet20}
for c in ${PROF_CASES:-bf16:256 bf16:1024}; do
  dt=${c%%:*}; b=${c##*:}
  d=gpurun_out/prof_${MODEL}_${dt}_b${b}
  rm -rf $d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- \
    python3 tools/bench_forward.py --model $MODEL --dtype $dt --batches $b --iters 20 \
    > $d.log 2>&1 || { echo "FAILED $c"; tail -5 $d.log; exit 1; }
  grep '^{' $d.log
  python3 tools/prof_summary.py $(find $d -name '*.db' | head -1) --top 12 > $d.txt
  cat $d.txt
done
