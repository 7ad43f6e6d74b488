#!/bin/bash
# GPU-box: GPU tests, default bench, then a rocprofv3 kernel-trace of a short bench run.
# Extra bench args come from BENCH_ARGS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof
GALE_ROCTX=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d gpurun_out/prof -o run -- \
  python3 bench.py --steps 50 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/prof_bench.log
python3 tools/prof_summary.py $(find gpurun_out/prof -name '*.db' | head -1) > gpurun_out/prof_bench.txt
cat gpurun_out/prof_bench.txt
exit $rc
