"""GPU-only forward throughput of a model replica (hipGraph replay), for kernel work.

Not the headline metric (that is bench.py: end-to-end Kafka -> JSON -> GPU -> JSON -> Kafka).
"""

import argparse
import json
import os
import sys
import time

sys.path.append(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from gale.models import get_model  # noqa: E402
from gale.parallel.weights import materialize_weights  # noqa: E402
from gale.runtime.replica import ModelReplica  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet20")
    ap.add_argument("--batches", default="1,64,256,1024,4096")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--conv-path", type=int, default=0,
                    help="0 auto, 1 conv_mfma only, 2 GEMM conv wherever the shape allows")
    ap.add_argument("--streams", type=int, default=1,
                    help="batches in flight at once, one replica slot and HIP stream each (the "
                         "serving engine keeps 2 per replica): whole-GPU throughput when a "
                         "memory-bound layer of one batch overlaps a compute-bound one of another")
    ap.add_argument("--chunk", default="",
                    help="LAYER:N - layers before LAYER run per chunk of N images "
                         "(PlanSpec::chunk_ops)")
    ap.add_argument("--no-fuse-blocks", action="store_true",
                    help="run the ResNet-50 56x56 bottlenecks layer by layer (A/B of "
                         "bottleneck_fused.hip)")
    a = ap.parse_args()
    from gale._native import native
    native().set_conv_path(a.conv_path)
    net = get_model(a.model)
    dev = torch.device("cuda", 0)
    packed = materialize_weights(net, dev, wdtype=a.dtype)
    bs = [int(b) for b in a.batches.split(",")]
    chunk = None
    if a.chunk:
        name, n = a.chunk.split(":")
        chunk = ([L.name for L in net.layers].index(name), int(n))
    ns = max(1, a.streams)
    rep = ModelReplica(net, packed, max_batch=max(bs), slots=ns, buckets=bs, wdtype=a.dtype,
                       chunk=chunk, fuse_blocks=not a.no_fuse_blocks)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(ns - 1)]
    ss = [st.cuda_stream for st in streams]
    res = []
    for b in bs:
        for _ in range(3):
            for k in range(ns):
                rep.executor.run(k, b, ss[k], not a.eager)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            for k in range(ns):
                rep.executor.run(k, b, ss[k], not a.eager)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.iters / ns  # per batch
        flops = 2 * net.macs_per_image() * b
        r = dict(model=a.model, dtype=a.dtype, conv_path=a.conv_path, batch=b, ms=dt * 1e3,
                 img_s=b / dt, tflops=flops / dt / 1e12, graph=not a.eager, chunk=a.chunk,
                 streams=ns, fuse_blocks=not a.no_fuse_blocks)
        res.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
