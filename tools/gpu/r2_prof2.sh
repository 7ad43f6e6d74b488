# e2e rocprofv3 kernel stats of the default bench (GPU ingest + GPU text); a second pass without
# GPU ingest only if the first fails
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_e2e2
if timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e2e2 -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_e2e2.log 2>&1; then
  python3 tools/prof_summary.py $(find gpurun_out/prof_e2e2 -name '*.db' | head -1) --top 14 > gpurun_out/r2_prof_e2e2.txt 2>&1
  cat gpurun_out/r2_prof_e2e2.txt; tail -1 gpurun_out/prof_e2e2.log | cut -c1-300
else
  echo "FIRST PASS FAILED rc=$?"; grep -v "^    @" gpurun_out/prof_e2e2.log | tail -8
fi
