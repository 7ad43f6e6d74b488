#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): whole-node images/s + p50 latency of the streaming
inference topology, CIFAR-10 ResNet-20 bf16, one data-parallel replica per GPU.

What one rank (= one GPU, launched by torch.distributed.run for N > 1) does:

* starts an embedded Kafka-protocol broker on 127.0.0.1 (one Kafka partition per replica,
  BASELINE config 3) and preloads its input topic with synthetic InstObj records
  ``{"instances": [[[[...32x32x3 Java-formatted floats...]]]]}`` (~35 KB of JSON per image);
* initialises ResNet-20 weights on rank 0 (seeded random init) and RCCL-broadcasts the packed
  buffer over xGMI to every other rank;
* runs the full gale engine: Kafka Fetch over TCP -> envelope scan -> micro-batcher -> pinned
  staging -> H2D -> GPU JSON parse -> hipGraph ResNet-20 forward -> D2H softmax ->
  {"predictions": ...} encode -> Kafka Produce (acks=1) -> ack.

A "step" is one micro-batch per replica, i.e. ``--batch x --replicas-per-gpu`` images per GPU
completing that whole path (acknowledged by the broker). W warmup
steps run first (graphs are captured before that), then exactly K timed steps, bracketed by a
barrier + ``torch.cuda.synchronize()``. ``value`` is the whole-job aggregate images/s (sum over
ranks of timed images / the slowest rank's time). p50 latency = median time from a record's
fetch to its output record's produce-ack, over all timed records of rank 0 (queue included).
"""

from __future__ import annotations

import argparse
import json
import os
import resource
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec (whole node) + p50 latency, CIFAR-10 ResNet-20 at 1/2/4/8 GPUs"


def parse_args():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="resnet20", choices=["lenet5", "resnet20", "resnet50"])
    ap.add_argument("--batch", type=int, default=256, help="images per micro-batch (max_batch)")
    ap.add_argument("--images-per-record", type=int, default=1)
    ap.add_argument("--distinct", type=int, default=1024, help="distinct synthetic images")
    ap.add_argument("--partitions", type=int, default=0,
                    help="input partitions per GPU (default: one per replica, BASELINE config 3)")
    ap.add_argument("--source-parallelism", type=int, default=0,
                    help="consumer threads (default: one per partition)")
    ap.add_argument("--sink-parallelism", type=int, default=2)
    ap.add_argument("--decode-threads", type=int, default=2)
    ap.add_argument("--replicas-per-gpu", type=int, default=0,
                    help="model replicas (streams) per GPU, each with its own input partition "
                         "(0 = from the host CPU share: 4 with >= 16 cores per GPU)")
    ap.add_argument("--max-wait-us", type=int, default=2000)
    ap.add_argument("--queue-batches", type=int, default=4,
                    help="records buffered in the engine, in units of --batch")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--stub", action="store_true", help="CPU stub replicas (no GPU)")
    ap.add_argument("--stub-null", action="store_true",
                    help="stub replicas skip parsing (measures the host Kafka/codec path only)")
    ap.add_argument("--check-crcs", action=argparse.BooleanOptionalAction, default=True,
                    help="consumer CRC32C verification (Kafka check.crcs; diagnosis only)")
    ap.add_argument("--rate", type=float, default=0.0,
                    help="offered load in images/s per GPU: records are appended to the broker "
                         "at this rate while the engine runs (latency under load, BASELINE "
                         "config 5); 0 = a preloaded backlog (maximum throughput)")
    ap.add_argument("--broker-zero-copy", action=argparse.BooleanOptionalAction, default=False,
                    help="embedded broker sends fetched batches with vmsplice/splice (Kafka's "
                         "sendfile analogue) instead of writev copies")
    ap.add_argument("--numa-pin", action=argparse.BooleanOptionalAction, default=True,
                    help="pin the host pipeline's threads to the GPU's NUMA node")
    ap.add_argument("--cpus-per-rank", type=int, default=0,
                    help="with --numa-pin: only this rank's slice of the node's CPUs (0 = all)")
    ap.add_argument("--timeout", type=float, default=600.0)
    return ap.parse_args()


class RateFeeder:
    """Appends pre-encoded record batches (by reference) to the input partitions at a fixed
    image rate from a background thread: an open-loop load generator, so latency is measured
    at a known offered load instead of against a backlog."""

    def __init__(self, broker, topic, parts, batches, images_per_batch, rate):
        import threading

        self.broker, self.topic, self.parts, self.batches = broker, topic, parts, batches
        self.ipb, self.rate = images_per_batch, rate
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="rate-feeder", daemon=True)

    def _run(self):
        t0 = time.perf_counter()
        sent = 0
        i = 0
        while not self._stop.is_set():
            due = (time.perf_counter() - t0) * self.rate
            while sent + self.ipb <= due:
                self.broker.append_batch_repeated(self.topic, i % self.parts,
                                                  self.batches[i % len(self.batches)], 1)
                sent += self.ipb
                i += 1
            time.sleep(0.0002)

    def start(self):
        self._t.start()

    def stop(self):
        self._stop.set()
        self._t.join()


def main() -> int:
    a = parse_args()
    if a.replicas_per_gpu <= 0:
        # the host pipeline (Kafka fetch + CRC + scan + encode + produce, and the embedded
        # broker of this rank) needs ~3 cores per replica at full rate
        from gale.utils import host_cpus_per_rank

        a.replicas_per_gpu = max(1, min(4, int(host_cpus_per_rank() // 4)))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    use_gpu = not a.stub
    if use_gpu and not torch.cuda.is_available():
        raise SystemExit("bench.py: no GPU visible (use --stub for the CPU plumbing run)")
    if use_gpu:
        torch.cuda.set_device(local_rank)
        if a.numa_pin:
            from gale.utils import pin_to_gpu_numa

            pin_to_gpu_numa(local_rank, a.cpus_per_rank)
    if world > 1:
        dist.init_process_group(backend="nccl" if use_gpu else "gloo",
                                device_id=torch.device("cuda", local_rank) if use_gpu else None)

    from gale._native import native
    from gale.config import GaleConfig
    from gale.data import encode_batches, encode_records, preload, synthetic_images
    from gale.engine import Engine
    from gale.models import get_model

    net = get_model(a.model)
    K = native().kafka
    ipr = a.images_per_record
    parts = a.partitions or a.replicas_per_gpu
    # records per preloaded RecordBatch (rate mode: small batches, arrivals are not bursty)
    # (the feeder thread keeps to ~10k appends/s)
    rpb = min(64, max(8, int(a.rate // 10000))) if a.rate > 0 else 64
    # ... and at most ~4 MB per RecordBatch, as a producer's batch.size would keep it: a fetch
    # always returns at least one whole batch (KIP-74), so 64 ResNet-50 records (1.7 MB each)
    # in one batch would turn every fetch into a 109 MB response
    rec_bytes = 12 * int(np.prod(net.input_shape)) * ipr  # ~Java float text per record
    rpb = max(1, min(rpb, (4 << 20) // rec_bytes))
    broker = K.Broker(max_message_bytes=256 << 20, retention_bytes=1 << 62,
                      zero_copy=a.broker_zero_copy)
    broker.start()
    broker.create_topic("gale-in", parts)
    broker.create_topic("gale-out", 1)
    # slack: the pipeline keeps fetching past the timed window until stop() (records are
    # appended by reference, so generous slack costs no memory)
    step_images = a.batch * a.replicas_per_gpu  # one micro-batch per replica
    per_rank_images = ((a.warmup + a.steps + 4) * step_images + 8192 * ipr
                       + 4 * a.queue_batches * a.batch + parts * 1024 * ipr)
    n_records = -(-per_rank_images // ipr)
    distinct = max(rpb, (a.distinct // (ipr * rpb)) * rpb) * ipr
    imgs = synthetic_images(distinct, net.input_shape, seed=1234 + rank)
    batches = encode_batches(encode_records(imgs, ipr), rpb)
    if a.rate <= 0:
        for p in range(parts):
            preload(broker, "gale-in", p, batches, -(-n_records // parts), rpb)
    del imgs
    feeder = None
    if a.rate > 0:
        feeder = RateFeeder(broker, "gale-in", parts, batches, rpb * ipr, a.rate)

    cfg = GaleConfig(topology_name=f"bench-r{rank}", input_topic="gale-in",
                     output_topic="gale-out", bootstrap=f"127.0.0.1:{broker.port}",
                     group_id="bench", start_offset="earliest", model=a.model, dtype=a.dtype,
                     max_batch=a.batch, max_wait_us=a.max_wait_us,
                     queue_depth=max(1, a.queue_batches * a.batch // ipr),
                     source_parallelism=a.source_parallelism or parts,
                     sink_parallelism=a.sink_parallelism, replicas=a.replicas_per_gpu,
                     decode_threads=a.decode_threads,
                     stub=a.stub, stub_null=a.stub_null, commit_interval_ms=500,
                     check_crcs=a.check_crcs)
    devices = [local_rank] if use_gpu else None
    warm_records = -(-max(1, a.warmup) * step_images // ipr)
    timed_records = -(-a.steps * step_images // ipr)
    # ONE engine: warm-up and timed window are the same steady-state pipeline (connections,
    # pinned fetch buffers, captured graphs all warm); the timed window starts at a barrier
    # once every rank has completed its warm-up records and ends when K more steps completed.
    eng = Engine(cfg, devices=devices)  # weights: seeded on rank 0, RCCL-broadcast
    eng.start()
    if feeder:
        feeder.start()
    if not eng.wait_completed(warm_records, a.timeout):
        raise SystemExit(f"rank {rank}: warm-up timed out ({eng.completed}/{warm_records})")
    warm_done = eng.completed
    if world > 1:
        dist.barrier()
    if use_gpu:
        torch.cuda.synchronize()
    eng.reset_stats()
    c0 = eng.completed
    t0 = time.perf_counter()
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    reached = eng.wait_completed(c0 + timed_records, a.timeout)
    if use_gpu:
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    done_records = eng.completed - c0
    cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    st = eng.stats()
    if world > 1:
        dist.barrier()
    if feeder:
        feeder.stop()
    eng.stop()
    broker.stop()
    if not reached:
        raise SystemExit(f"rank {rank}: timed out after {elapsed:.1f}s "
                         f"({done_records}/{timed_records} records)")
    images = done_records * ipr  # >= K steps (completions arrive a micro-batch at a time)
    t = torch.tensor([elapsed, float(images)], dtype=torch.float64)
    if world > 1:
        tt = t.cuda() if use_gpu else t
        mx = tt.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tt.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed_max, total_images = float(mx[0]), float(sm[1])
    else:
        elapsed_max, total_images = elapsed, float(images)
    if rank == 0:
        value = total_images / elapsed_max
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "images/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup,
            # time per step-equivalent of completed work (>= K steps completed in the window)
            "ms_per_step": round(elapsed_max / (total_images / (step_images * world)) * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
            "data": f"synthetic (uniform [0,1) {'x'.join(map(str, net.input_shape))} InstObj "
                    "JSON records, Java float format, preloaded into an embedded Kafka-protocol "
                    "broker); random-init weights (seed 0) RCCL-broadcast from rank 0",
            "config": {"model": a.model, "global_batch": step_images * world, "seq_len": None,
                       "parallelism": f"dp{world}", "images_per_record": ipr,
                       "max_wait_us": a.max_wait_us, "replicas_per_gpu": a.replicas_per_gpu,
                       "path": "kafka-fetch->gpu-json-parse->hipgraph-forward->kafka-produce"},
            "load": (f"offered {a.rate:.0f} images/s per GPU" if a.rate > 0
                     else "preloaded backlog (max throughput; latency includes queueing)"),
            "p50_latency_ms": round(st["e2e_us_p50"] / 1e3, 3),
            "p99_latency_ms": round(st["e2e_us_p99"] / 1e3, 3),
            "device_ms_p50": round(st["device_us_p50"] / 1e3, 3),
            "batch_images_mean": round(st["batch_images_mean"], 1),
            "json_mb_per_s_rank0": round(st["bytes_in"] / elapsed / 1e6, 1),
            "cpu_cores_busy_rank0": round(cpu_s / elapsed, 2),
            "warmup_records": warm_done,
            "rank0_thread_s": {k[9:]: round(v, 3) for k, v in st.items()
                               if k.startswith("thread_s_")},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
