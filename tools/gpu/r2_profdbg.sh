# which part of the e2e path makes the bench crash under rocprofv3 --kernel-trace?
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for args in "--no-gpu-ingest" "--decode-threads 1" "--no-gpu-encode"; do
  tag=$(echo $args | tr -d ' -')
  rm -rf gpurun_out/pd_$tag
  if timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pd_$tag -o run -- python3 bench.py --steps 5 --warmup 2 $args > gpurun_out/pd_$tag.log 2>&1; then
    echo "OK $args"; python3 tools/prof_summary.py $(find gpurun_out/pd_$tag -name '*.db' | head -1) --top 8 2>&1 | cut -c1-160
  else
    echo "FAIL($?) $args"; grep -m3 "SIGSEGV\|Aborted\|gale::" gpurun_out/pd_$tag.log
  fi
done
