#!/bin/bash
# which native threads of a bench run burn CPU: tid, name, wchan, CPU ticks at two instants 5 s
# apart (sampled mid-run); extra bench args from $1 (label) and the rest
set -o pipefail
label=${1:-def}; shift
mkdir -p gpurun_out/threads
python3 bench.py --steps 400 --warmup 5 --latency-load 0 "$@" > gpurun_out/threads/b_$label.json 2> gpurun_out/threads/b_$label.err &
pid=$!
sleep 16
snap() {
  for t in /proc/$pid/task/*; do
    echo "$(basename $t) $(cat $t/comm | tr ' ' '_') $(cat $t/wchan 2>/dev/null) $(awk '{print $14+$15}' $t/stat)"
  done
}
snap > gpurun_out/threads/s1_$label.txt
sleep 5
snap > gpurun_out/threads/s2_$label.txt
( sleep 120; kill $pid 2>/dev/null ) &
wait $pid
