# per-process multi-rank path with real GPU replicas (torchrun world 2 sharing the one GPU of the
# box, gloo process group): broker cluster, shared input topic, weight broadcast, max-over-ranks
# timing. Launched from bash, not from a GPU-initialised pytest process (no fork+exec from it).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --shared-gpu-rehearsal \
  --steps 4 --warmup 1 --distinct 2048 --step-images 8192 --replicas-per-gpu 3 --partitions 6 \
  --decode-threads 2 --min-warmup-s 0.5 --no-numa-pin --timeout 90 \
  > gpurun_out/rehearsal.json 2> gpurun_out/rehearsal.err || { tail -30 gpurun_out/rehearsal.err; exit 1; }
python -c "
import json
r = [json.loads(x) for x in open('gpurun_out/rehearsal.json') if x.startswith('{')]
assert len(r) == 1, r
r = r[0]
assert r['n_gpus'] == 2 and r['config']['parallelism'] == 'dp2' and r['value'] > 0, r
print('REHEARSAL_OK', r['value'], r['config']['partitions'], r['batch_images_mean'])
"
