#!/bin/bash
# which native threads of a bench run burn CPU: tid, name, wchan, current syscall, CPU ticks at
# two instants 5 s apart (sampled mid-run)
set -o pipefail
mkdir -p gpurun_out/threads
python3 bench.py --steps 60 --warmup 5 --latency-load 0 > gpurun_out/threads/b.json 2> gpurun_out/threads/b.err &
pid=$!
sleep 22
snap() {
  for t in /proc/$pid/task/*; do
    echo "$(basename $t) $(cat $t/comm | tr ' ' '_') $(cat $t/wchan 2>/dev/null) $(cut -d' ' -f1 $t/syscall 2>/dev/null) $(awk '{print $14+$15}' $t/stat)"
  done
}
snap > gpurun_out/threads/s1.txt
sleep 5
snap > gpurun_out/threads/s2.txt
( sleep 120; kill $pid 2>/dev/null ) &
wait $pid
