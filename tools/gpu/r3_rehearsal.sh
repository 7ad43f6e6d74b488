#!/bin/bash
# per-process multi-rank rehearsal on the one-GPU box: torchrun world 2 and 4 sharing the GPU
# (gloo group, --shared-gpu-rehearsal), full-size steps, latency phase gathered over ranks
set -o pipefail
d=gpurun_out/rehearsal
mkdir -p $d
export TMPDIR=/tmp
for w in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node $w \
    --master-addr 127.0.0.1 --master-port $((29560 + w)) bench.py --gpus 1 --shared-gpu-rehearsal \
    --steps 10 --warmup 3 > $d/w$w.log 2>&1 || { tail -30 $d/w$w.log; exit 1; }
  grep '^{' $d/w$w.log | tail -1 | cut -c1-400
done
