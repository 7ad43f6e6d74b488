#!/bin/bash
# GPU-box: rocprofv3 kernel + roctx marker trace of one bench.py run (args from BENCH_ARGS);
# writes the kernel / range summary and a per-thread range timeline sample.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_e2e
GALE_ROCTX=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d gpurun_out/prof_e2e -o run -- \
  python3 bench.py ${BENCH_ARGS:-} > gpurun_out/prof_e2e.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/prof_e2e.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py $(find gpurun_out/prof_e2e -name '*.db' | head -1) > gpurun_out/prof_e2e.txt
cat gpurun_out/prof_e2e.txt
