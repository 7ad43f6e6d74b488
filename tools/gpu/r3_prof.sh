#!/bin/bash
# rocprofv3 kernel trace of the DEFAULT serving configuration (bench.py defaults, short run);
# the native crash reporter prints a backtrace if anything faults under the tool
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_def
GPU_MAX_HW_QUEUES=32 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_def -o run -- \
  python3 bench.py --steps 10 --warmup 3 --latency-load 0 > gpurun_out/prof_def.log 2>&1
rc=$?; echo "prof rc=$rc"; grep -A30 "gale crash" gpurun_out/prof_def.log | head -60
tail -1 gpurun_out/prof_def.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py $(find gpurun_out/prof_def -name '*.db' | head -1) --top 12 > gpurun_out/prof_def.txt 2>&1
cat gpurun_out/prof_def.txt
