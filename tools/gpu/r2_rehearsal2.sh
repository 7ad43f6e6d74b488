# per-process rehearsal (world 2 on one GPU): outputs to the rank's own partition vs round-robin
set -o pipefail
mkdir -p gpurun_out
for lo in --local-output --no-local-output --local-output --no-local-output; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --shared-gpu-rehearsal \
    --steps 10 --warmup 1 --distinct 4096 --step-images 16384 --replicas-per-gpu 3 --partitions 6 \
    --decode-threads 2 --min-warmup-s 1 --no-numa-pin --timeout 90 $lo \
    > gpurun_out/rehearsal.json 2> gpurun_out/rehearsal.err || { tail -30 gpurun_out/rehearsal.err; exit 1; }
  python -c "
import json
r = [json.loads(x) for x in open('gpurun_out/rehearsal.json') if x.startswith('{')][0]
print('$lo', r['value'], r['timed_s'], r['cpu_cores_by_stage_rank0'])
"
done
