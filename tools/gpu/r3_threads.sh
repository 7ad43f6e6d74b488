#!/bin/bash
# which native threads of a bench run burn CPU: name, tid, wchan, CPU seconds (sampled mid-run)
set -o pipefail
mkdir -p gpurun_out/threads
timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --timeline gpurun_out/threads/tl.jsonl > gpurun_out/threads/b.json 2> gpurun_out/threads/b.err &
pid=$!
sleep 25
for t in /proc/$pid/task/*; do
  echo "$(basename $t) $(cat $t/comm) $(cat $t/wchan 2>/dev/null) $(awk '{print $14+$15}' $t/stat)"
done | sort -k4 -n -r | head -40 > gpurun_out/threads/tasks.txt
wait $pid
