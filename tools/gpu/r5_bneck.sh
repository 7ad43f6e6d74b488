#!/bin/bash
# Fused 56x56 bottleneck (bottleneck_fused.hip): GPU tests, forward A/B (layered vs fused, x2
# interleaved) and a kernel trace of the fused forward.
set -o pipefail
d=gpurun_out/bneck
mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 120 python tools/bench_bneck.py --layered > $d/kern.jsonl 2>&1 && cat $d/kern.jsonl &&
timeout -k 10 300 python -u -m pytest tests/test_bottleneck_gpu.py -x -v --timeout 120 \
    --timeout-method thread > $d/pytest.log 2>&1 || { tail -40 $d/pytest.log; exit 1; }
tail -5 $d/pytest.log
for r in 1 2; do
  for f in "--no-fuse-blocks" "" "--no-fuse-blocks --streams 2" "--streams 2"; do
    timeout -k 10 200 python tools/bench_forward.py --model resnet50 --batches 256 --iters 30 $f \
        >> $d/ab.jsonl 2> $d/ab.err || { tail -20 $d/ab.err; exit 1; }
  done
done
cat $d/ab.jsonl
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d/prof -o run -- \
    python tools/bench_forward.py --model resnet50 --batches 256 --iters 20 > $d/fwd.log 2>&1 || exit 1
db=$(find $d/prof -name '*.db' | head -1)
if [ -n "$db" ]; then python tools/prof_summary.py $db --by-grid --top 40 > $d/by_grid.txt; fi
st=$(find $d/prof -name '*kernel_stats.csv' | head -1)
[ -n "$st" ] && cp $st $d/kernel_stats.csv
head -30 $d/by_grid.txt 2>/dev/null
rm -rf $d/prof
