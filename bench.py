#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): whole-node images/s + p50 latency of the streaming
inference topology, CIFAR-10 ResNet-20 bf16, one data-parallel replica group per GPU.

What one rank (= one GPU, launched by torch.distributed.run for N > 1) does:

* starts an embedded Kafka-protocol broker on 127.0.0.1. With N ranks the N brokers form ONE
  Kafka cluster: the input topic has N x P partitions, partition p led by rank p % N's broker,
  and every rank consumes exactly the partitions it leads - so all ranks share one input topic,
  as the reference's spouts share INPUT_TOPIC. P (--partitions) defaults to 11-12 per GPU, one
  consumer thread each (more TCP connections than one core can receive on; size_pipeline).
  ``--baseline-config 3`` runs BASELINE config 3 literally: ONE partition per GPU data-parallel
  replica, consumed by one source thread (MainTopology.java:26-27,61-62 map 2 spouts to 4 bolts;
  the replica's streams still share that partition's records);
* feeds the input partitions with synthetic InstObj records ``{"instances": [[[[...]]]]}``
  (32x32x3 Java-formatted floats, ~35 KB of JSON per image) drawn from ``--distinct`` distinct
  images (default 65536, ~2.3 GB of JSON, so the host stages stream from DRAM, not from cache).
  The pre-encoded batches are appended by reference and kept topped up ahead of the consumers;
  the broker stamps them with LogAppendTime, so record end-to-end latency (append -> produce
  ack) is measured exactly;
* initialises ResNet-20 weights on rank 0 (seeded random init) and RCCL-broadcasts the packed
  buffer over xGMI to every other rank;
* runs the full gale engine: Kafka Fetch over TCP (each body received through a cache-resident
  window and nibble-packed into pinned memory) -> GPU ingest (CRC32C + image counts, one kernel
  per fetch) -> micro-batcher -> per batch step, launched kernel by kernel (--step-launch direct,
  the default; a hipGraph replay is --step-launch graph): GPU JSON parse -> whole-network
  ResNet-20 forward whose epilogue writes the softmax AND its {"predictions": ...} text into
  host-mapped memory -> Kafka Produce (acks=1) -> ack.

Steady state: warm-up is W steps AND at least ``--min-warmup-s`` seconds AND until the last
four 500 ms rate windows (2 s) all lie within 5 % of their mean (capped at ``--max-warmup-s``). A step is
``--step-images`` images per GPU (default 262144: 1024 micro-batches of 256) completing the whole
path (acknowledged by the broker), so the default K = 20 steps is a ~3.5 s window on one
MI355X at 1.5 M img/s (65536-image steps fell below 1 s once the pipeline passed 1.5 M img/s;
131072-image steps let single host hiccups swing a step's rate by 10-20 %). The K timed steps are bracketed by a barrier + ``torch.cuda.synchronize()``; ``value``
is the whole-job images/s (sum over ranks of the images completed in the window / the slowest
rank's window). The per-step rates give the within-run spread.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec (whole node) + p50 latency, CIFAR-10 ResNet-20 at 1/2/4/8 GPUs"
# the headline metric is BASELINE.json's (ResNet-20); the other BASELINE configs report the same
# quantity under their own model's name
METRICS = {"resnet20": METRIC,
           "lenet5": "images/sec (whole node) + p50 latency, MNIST LeNet-5",
           "resnet50": "images/sec (whole node) + p50 latency, ImageNet ResNet-50"}


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--step-images", type=int, default=0,
                    help="images per GPU per step (the unit of --steps / --warmup); default "
                         "262144 (4096 for resnet50)")
    ap.add_argument("--min-warmup-s", type=float, default=2.0)
    ap.add_argument("--max-warmup-s", type=float, default=20.0)
    ap.add_argument("--model", default="resnet20", choices=["lenet5", "resnet20", "resnet50"])
    ap.add_argument("--batch", type=int, default=0,
                    help="images per micro-batch (max_batch; default 256, 128 for resnet50)")
    ap.add_argument("--images-per-record", type=int, default=1)
    ap.add_argument("--distinct", type=int, default=0,
                    help="distinct synthetic images (default 65536; 256 = 435 MB for resnet50)")
    ap.add_argument("--partitions", type=int, default=0,
                    help="input partitions per GPU (default 11-12 with >= 16 host CPUs per GPU, "
                         "see size_pipeline)")
    ap.add_argument("--baseline-config", type=int, default=0, choices=[0, 3],
                    help="3 = BASELINE config 3 as written: one input partition per GPU "
                         "data-parallel replica, one source thread per partition")
    ap.add_argument("--source-parallelism", type=int, default=0,
                    help="consumer threads (default: one per partition)")
    ap.add_argument("--sink-parallelism", type=int, default=2)
    ap.add_argument("--decode-threads", type=int, default=0,
                    help="GPU-ingest / decode workers (0 = from the host CPU share)")
    ap.add_argument("--replicas-per-gpu", type=int, default=0,
                    help="model replicas (streams) per GPU (0 = from the host CPU share: 6 "
                         "with >= 16 cores per GPU, else ~1 per 4 cores, at most 4)")
    ap.add_argument("--max-wait-us", type=int, default=-1,
                    help="micro-batch wait (default 2000; 20000 for resnet50)")
    ap.add_argument("--queue-batches", type=int, default=4,
                    help="records buffered in the engine, in units of --batch")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8", "fp32"])
    ap.add_argument("--slo-p99-ms", type=float, default=0.0,
                    help="latency-SLO mode: adapt the batch/wait bound to keep p99 under this")
    ap.add_argument("--stub", action="store_true", help="CPU stub replicas (no GPU)")
    ap.add_argument("--stub-null", action="store_true",
                    help="stub replicas skip parsing (measures the host Kafka/codec path only)")
    ap.add_argument("--gpu-encode", action=argparse.BooleanOptionalAction, default=True,
                    help="format the prediction text (Java Float.toString) on the GPU")
    ap.add_argument("--graph", action=argparse.BooleanOptionalAction, default=True,
                    help="replay each batch's forward as a captured hipGraph (else eager)")
    ap.add_argument("--graph-step", action=argparse.BooleanOptionalAction, default=True,
                    help="run each batch step (metadata H2D, parse, forward, format, status D2H) "
                         "as one replay of a captured per-slot hipGraph (whole-network plans)")
    ap.add_argument("--gpu-ingest", action=argparse.BooleanOptionalAction, default=True,
                    help="CRC32C + image counting of fetch buffers on the GPU (host reads only "
                         "Kafka framing)")
    ap.add_argument("--text-pack", action=argparse.BooleanOptionalAction, default=True,
                    help="sources nibble-pack the fetched JSON text for the host->GPU link "
                         "through a cache-resident receive window (expanded on the device; needs "
                         "AVX-512 VBMI): half the link and pinned-memory bytes, "
                         "profiles/archive/r4_ab_step_graph_text_pack.jsonl")
    ap.add_argument("--pack-nt", action=argparse.BooleanOptionalAction, default=True,
                    help="the sources write the packed text with non-temporal stores (no "
                         "read-for-ownership of the pinned destination lines, the receive window "
                         "stays in L2)")
    ap.add_argument("--pinned-fetch-mb", type=int, default=4096,
                    help="pinned fetch-buffer budget per GPU (doubled with --text-pack)")
    ap.add_argument("--text-pack-window-kb", type=int, default=256,
                    help="bounce receive window per source thread")
    ap.add_argument("--ingest-parse", action=argparse.BooleanOptionalAction, default=True,
                    help="the GPU ingest parses each fetch's records into an fp32 image arena, "
                         "so the batch step runs the forward only (whole-network plans)")
    ap.add_argument("--text-pack-bounce", action=argparse.BooleanOptionalAction, default=True,
                    help="with --text-pack: receive through a cache-resident window, keep only "
                         "the packed text + a sparse framing copy in pinned memory")
    ap.add_argument("--check-crcs", action=argparse.BooleanOptionalAction, default=True,
                    help="consumer CRC32C verification (Kafka check.crcs; diagnosis only)")
    ap.add_argument("--rate", type=float, default=0.0,
                    help="offered load in images/s per GPU: records are appended to the broker "
                         "at this rate while the engine runs (latency under load, BASELINE "
                         "config 5); 0 = a backlog kept ahead of the consumers (max throughput)")
    # zero-copy fetch responses, as a Kafka broker serves them (sendfile from the page cache):
    # one host copy less per byte. On boxes whose memory system is loaded it is the difference
    # between 0.98 M (copying, CPU-bound at 16 of 16 cores) and 1.43-1.52 M img/s; on quiet
    # boxes both sit near the link (profiles/archive/r3_broker_zero_copy_default.jsonl)
    ap.add_argument("--broker-zero-copy", action=argparse.BooleanOptionalAction, default=True,
                    help="embedded broker sends fetched batches with vmsplice/splice (Kafka's "
                         "sendfile analogue) instead of writev copies")
    ap.add_argument("--numa-pin", action=argparse.BooleanOptionalAction, default=True,
                    help="pin the host pipeline's threads to the GPU's NUMA node")
    ap.add_argument("--cpus-per-rank", type=int, default=0,
                    help="with --numa-pin: only this rank's slice of the node's CPUs (0 = the "
                         "whole NUMA node at N = 1, the rank's --rank-slices share at N > 1; "
                         "-1 = as many CPUs as the rank's cgroup CPU quota). Round-4 code on a "
                         "16-CPU-quota box, 3 interleaved runs each: whole node 2.08 M img/s, "
                         "16 physical cores 1.83 M (88 %%), 16 cores + SMT siblings 1.78 M "
                         "(85 %%; profiles/r5_slices_ab.jsonl)")
    ap.add_argument("--rank-slices", action=argparse.BooleanOptionalAction, default=False,
                    help="N > 1 with --cpus-per-rank 0: each rank gets a disjoint slice of its "
                         "GPU's NUMA node (the node's CPUs split evenly among the ranks on it, "
                         "whole cores with their SMT siblings: 16 + 16 per rank with 4 GPUs per "
                         "64-core socket) instead of every rank floating over the whole node. "
                         "Off by default: the 2-rank rehearsal on one box ran 3.6 %% slower with "
                         "slices (profiles/r5_rehearsal_world2_slices.jsonl), so no win is shown")
    ap.add_argument("--slice-smt", action="store_true",
                    help="with --cpus-per-rank N: the slice is N/2 whole physical cores with "
                         "their SMT siblings (what each of 4 ranks owns on a 64-core socket), "
                         "not the N lowest CPU ids")
    ap.add_argument("--step-launch", default="direct", choices=["graph", "direct"],
                    help="the per-batch step (parse -> forward, text + verdicts in the forward's "
                         "epilogue) as direct kernel launches or as one hipGraph replay (the "
                         "replay kept a HIP runtime helper thread spinning at ~0.8 core: 2.10 vs "
                         "2.18 M img/s, profiles/r5_ab_step_launch.jsonl)")
    ap.add_argument("--replica-priority", default="normal", choices=["normal", "high"],
                    help="stream priority of the replicas' step graphs")
    ap.add_argument("--gpu-wait-poll-us", type=int, default=20,
                    help="replica workers sleep-poll batch completion every N us (0 = spin)")
    ap.add_argument("--encode-threads", type=int, default=0,
                    help="threads for encoding the synthetic records (0 = host CPU share)")
    ap.add_argument("--single-process", action="store_true",
                    help="one process drives all --gpus GPUs (one engine: per-GPU locality "
                         "slots with work stealing, weights RCCL-broadcast in-process) instead "
                         "of one torch.distributed rank per GPU")
    ap.add_argument("--locality-split", type=int, default=1,
                    help="locality slots per GPU in this process (each with its own sources, "
                         "batcher and pinned pool; idle slots steal and parse stolen text from "
                         "host-pinned memory): the single-process multi-GPU dispatch on one GPU")
    ap.add_argument("--shared-gpu-rehearsal", action="store_true",
                    help="multi-rank rehearsal on a box with fewer GPUs than ranks: rank r uses "
                         "GPU r %% device_count and the process group runs over gloo (RCCL refuses "
                         "two ranks on one GPU); every other part of the per-rank path is the "
                         "real one. Not a measurement")
    ap.add_argument("--producer-buffer-mb", type=int, default=32,
                    help="unsent output bytes per sink producer (Kafka buffer.memory)")
    ap.add_argument("--producer-request-kb", type=int, default=1024,
                    help="bytes per produce request (Kafka max.request.size)")
    ap.add_argument("--local-output", action=argparse.BooleanOptionalAction, default=True,
                    help="each rank produces its outputs to the output partition its own broker "
                         "leads (--output-partition RANK) instead of round-robin over every "
                         "rank's broker (the unkeyed default)")
    ap.add_argument("--all-stats", action="store_true",
                    help="add every engine statistic of rank 0 (queue / device / e2e quantiles, "
                         "lag, thread seconds) to the JSON line")
    ap.add_argument("--latency-load", type=float, default=0.8,
                    help="after the throughput window, offer this fraction of the measured "
                         "throughput at a fixed rate (native open-loop producer) and report "
                         "p50/p99 of record append -> produce ack at microsecond resolution "
                         "(BASELINE's latency half); 0 = skip (p50 is then fetch -> ack under "
                         "the backlog, i.e. mostly queueing)")
    ap.add_argument("--latency-warmup-s", type=float, default=1.0)
    ap.add_argument("--latency-batch-records", type=int, default=0,
                    help="records per producer batch in the latency phase (0 = the backlog's "
                         "batches, 64 records)")
    ap.add_argument("--fetch-min-bytes", type=int, default=1,
                    help="consumer fetch.min.bytes (Kafka default 1)")
    ap.add_argument("--recv-lowat-kb", type=int, default=-1,
                    help="consumer receive low-water mark per receive call (SO_RCVLOWAT): one "
                         "wake-up per this many KB of a fetch response; 0 = per segment, -1 = "
                         "the bounce window with the bounce receive (profiles/"
                         "r4_ab_recv_lowat.jsonl)")
    ap.add_argument("--ingest-dev-timing", type=int, default=16,
                    help="time every N-th GPU ingest fetch of each lane on the device (events: "
                         "H2D copies, count pass, parse; latency_ingest_device_us); 0 off")
    ap.add_argument("--partition-max-kb", type=int, default=8192,
                    help="consumer max.partition.fetch.bytes (KB): the most one partition's fetch "
                         "response carries - the records at its head wait for the whole of it")
    ap.add_argument("--fetch-max-wait-ms", type=int, default=20,
                    help="consumer fetch.max.wait.ms (long-poll bound when no data is there)")
    ap.add_argument("--latency-sweep", default="",
                    help="after the --latency-load phase, more latency phases at these offered "
                         "loads (comma list of fractions of the measured throughput), reported "
                         "as latency_sweep (config 5: max load meeting a p99 SLO)")
    ap.add_argument("--latency-repeat", type=int, default=1,
                    help="latency phases per --latency-sweep load")
    ap.add_argument("--latency-dump", default="",
                    help="save rank 0's per-record latencies and ack times (.npz) of the latency "
                         "phase, to place a tail in time against --timeline")
    ap.add_argument("--latency-s", type=float, default=2.0)
    ap.add_argument("--timeline", default="",
                    help="write a JSON line every --timeline-ms (completions, per-stage CPU, "
                         "cgroup throttling, RSS, queue depth, lag) to this file (rank 0)")
    ap.add_argument("--timeline-ms", type=int, default=100)
    ap.add_argument("--timeout", type=float, default=600.0)
    ap.add_argument("--print-config", action="store_true",
                    help="print the per-rank configuration (pipeline sizing, CPU slices) this "
                         "command would run, then exit without running it")
    return ap.parse_args(argv)


def _cgroup_cpu_stat() -> dict:
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (ln.split() for ln in f if ln.strip())}
    except (OSError, ValueError):
        return {}


_TCP_KEYS = ("RetransSegs", "TCPTimeouts", "TCPLossProbes", "PruneCalled", "RcvPruned",
             "TCPRcvQDrop", "TCPBacklogDrop", "TCPZeroWindowDrop", "TCPRcvCollapsed",
             "TCPWantZeroWindowAdv", "TCPToZeroWindowAdv", "TCPFromZeroWindowAdv",
             "DelayedACKs", "TCPSpuriousRTOs")


def _tcp_counters() -> dict:
    """Host TCP counters (/proc/net/snmp Tcp + /proc/net/netstat TcpExt) that explain loopback
    stalls: retransmission timeouts, receive-queue pruning / drops, zero-window episodes."""
    out = {}
    for path in ("/proc/net/snmp", "/proc/net/netstat"):
        try:
            with open(path) as f:
                lines = f.read().splitlines()
        except OSError:
            continue
        for names, vals in zip(lines[::2], lines[1::2]):
            if names.split(":")[0] not in ("Tcp", "TcpExt"):
                continue
            for k, v in zip(names.split()[1:], vals.split()[1:]):
                if k in _TCP_KEYS:
                    out[k] = int(v)
    try:  # per-CPU network backlog: packets dropped (a full backlog) and softirq squeezes
        with open("/proc/net/softnet_stat") as f:
            rows = [ln.split() for ln in f if ln.strip()]
        out["softnet_dropped"] = sum(int(r[1], 16) for r in rows)
        out["softnet_squeezed"] = sum(int(r[2], 16) for r in rows)
    except (OSError, ValueError, IndexError):
        pass
    return out


def _rss_mb() -> float:
    try:
        with open("/proc/self/statm") as f:
            return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE") / 2**20
    except (OSError, ValueError):
        return -1.0


class Timeline:
    """Diagnostic sampler (--timeline): one JSON line per interval with the completion rate,
    CPU cores per pipeline stage, cgroup CPU throttling, RSS and the engine's queue / lag, so
    a throughput dip can be lined up with what the host was doing at that moment."""

    def __init__(self, path, interval_ms, broker):
        from gale.utils import thread_cpu_by_thread, thread_cpu_seconds

        self.per_thread = thread_cpu_by_thread
        self.main_tid = threading.main_thread().native_id
        self.f = open(path, "w")
        self.dt = interval_ms / 1e3
        self.broker = broker
        self.cpu = thread_cpu_seconds
        self.engine = None
        self.phase = "warmup"
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="timeline", daemon=True)

    def start(self, engine):
        self.engine = engine
        self._t.start()

    def _run(self):
        from gale.utils import name_this_thread

        name_this_thread("py-timeline")
        t0 = time.perf_counter()
        prev_t, prev_c, prev_cpu, prev_cg = t0, self.engine.completed, self.cpu(), _cgroup_cpu_stat()
        prev_b = self.broker.stats() if self.broker is not None else None
        prev_th = self.per_thread()
        prev_busy = {}
        groups = ("gl-brk", "gl-src", "gl-dec", "gl-rep", "gl-sink", "gl-watchdog")
        while not self._stop.wait(self.dt):
            now, c, cpu, cg = time.perf_counter(), self.engine.completed, self.cpu(), _cgroup_cpu_stat()
            dt = now - prev_t
            st = self.engine.stats()
            busy = {k: st.get("thread_s_" + k, 0.0) for k in ("poll", "handoff", "decode", "wait")}
            row = {"t": round(now - t0, 3), "mono": round(now, 4), "phase": self.phase,
                   # engine thread-seconds per second in source polls, source hand-off waits
                   # (decode queue full), decode and replica completion waits
                   "busy": {k: round((v - prev_busy.get(k, 0.0)) / dt, 2) for k, v in busy.items()},
                   "rate": round((c - prev_c) / dt),
                   "cores": {k: round((cpu[k] - prev_cpu.get(k, 0.0)) / dt, 2) for k in cpu},
                   "rss_mb": round(_rss_mb()),
                   "queue": int(st.get("queue_records", 0)),
                   # sources waiting for a free pinned fetch chunk (ingest backpressure)
                   "pinned_waits": int(st.get("pinned_waits", 0)),
                   "pinned_wait_s": round(st.get("pinned_wait_s", 0.0), 4),
                   "batches": int(st.get("batches", 0)),
                   "lag": int(st.get("lag_records", 0)),
                   "fetch_lag": int(st.get("fetch_lag_records", 0))}
            if cg:
                row["throttled_ms"] = round((cg.get("throttled_usec", 0)
                                             - prev_cg.get("throttled_usec", 0)) / 1e3, 1)
                row["cg_cores"] = round((cg.get("usage_usec", 0)
                                         - prev_cg.get("usage_usec", 0)) / 1e6 / dt, 2)
            th = self.per_thread()
            other = {}
            for k, v in th.items():
                if not k[1].startswith(groups):
                    name = "main" if k[0] == self.main_tid else f"{k[1]}:{k[0]}"
                    other[name] = other.get(name, 0.0) + v - prev_th.get(k, 0.0)
            row["other_top"] = {k: round(v / dt, 2) for k, v in
                                sorted(other.items(), key=lambda kv: -kv[1])[:4] if v > 0}
            # what the busiest unnamed thread is doing (its current syscall and wait channel):
            # the HIP / HSA runtime's helper threads carry the process name
            busiest = max(other.items(), key=lambda kv: kv[1], default=(None, 0.0))[0]
            if busiest and ":" in busiest:
                tid = busiest.rsplit(":", 1)[1]
                probe = {}
                for f in ("syscall", "wchan"):
                    try:
                        with open(f"/proc/self/task/{tid}/{f}") as fh:
                            probe[f] = fh.read().split()[0] if f == "syscall" else fh.read()
                    except (OSError, IndexError):
                        pass
                row["other_probe"] = probe
            prev_th = th
            if prev_b is not None:
                b = self.broker.stats()
                row["brk_out_gbs"] = round((b["bytes_out"] - prev_b["bytes_out"]) / dt / 1e9, 2)
                row["brk_in_mbs"] = round((b["bytes_in"] - prev_b["bytes_in"]) / dt / 1e6, 1)
                prev_b = b
            self.f.write(json.dumps(row) + "\n")
            self.f.flush()
            prev_t, prev_c, prev_cpu, prev_cg, prev_busy = now, c, cpu, cg, busy

    def stop(self):
        self._stop.set()
        self._t.join()
        self.f.close()


class Feeder:
    """Keeps the rank's input partitions supplied from a native BatchSet (batches appended by
    reference). Backlog mode (rate = 0): tops every partition up to ``ahead`` records past the
    engine's fetch position, so the consumers never starve and the log never holds more than
    a bounded backlog. Rate mode: an open-loop generator appending at a fixed image rate."""

    def __init__(self, broker, topic, parts, bset, rate=0.0, ahead_records=0):
        self.broker, self.topic, self.parts, self.bset = broker, topic, list(parts), bset
        self.rate, self.ahead = rate, ahead_records
        self.rpb = max(1, bset.records // len(bset))
        self.ipb = self.rpb * bset.images_per_record
        self.engine = None
        self._next = 0
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="feeder", daemon=True)
        self.native_tid = None

    def fill(self, records_per_partition):
        for p in self.parts:
            n = -(-records_per_partition // self.rpb)
            self.broker.append_cycled(self.topic, p, self.bset, n, self._next)
            self._next += n

    def _run(self):
        from gale.utils import name_this_thread

        name_this_thread("py-feeder")
        if self.rate > 0:
            t0, sent, i = time.perf_counter(), 0, 0
            while not self._stop.is_set():
                due = (time.perf_counter() - t0) * self.rate
                while sent + self.ipb <= due:
                    self.broker.append_cycled(self.topic, self.parts[i % len(self.parts)],
                                              self.bset, 1, self._next)
                    self._next += 1
                    sent += self.ipb
                    i += 1
                time.sleep(0.0002)
            return
        while not self._stop.wait(0.005):
            eng = self.engine
            if eng is None:
                continue
            pos = {o["partition"]: o["fetched"] for o in eng.partition_offsets()}
            for p in self.parts:
                short = pos.get(p, 0) + self.ahead - self.broker.log_end(self.topic, p)
                if short > 0:
                    n = -(-short // self.rpb)
                    self.broker.append_cycled(self.topic, p, self.bset, n, self._next)
                    self._next += n

    def start(self, engine):
        self.engine = engine
        self._t.start()

    def stop(self):
        self._stop.set()
        self._t.join()


def warm_up(eng, records, a, rate_window=0.5, windows=4, tol=0.05):
    """W steps, then until >= min_warmup_s elapsed and the last ``windows`` rate windows of
    ``rate_window`` s (>= 2 s together) all lie within ``tol`` of their mean (or max_warmup_s).
    A slow oscillation (e.g. CFS throttling phases of ~0.5-1 s) shows up as a spread across
    the 2 s span, which two adjacent 250 ms windows could miss. Returns (seconds, rates)."""
    t_start = time.perf_counter()
    if not eng.wait_completed(records, a.timeout):
        raise SystemExit(f"warm-up timed out ({eng.completed}/{records})")
    rates = []
    while True:
        c0, t0 = eng.completed, time.perf_counter()
        time.sleep(rate_window)
        rates.append((eng.completed - c0) / (time.perf_counter() - t0))
        el = time.perf_counter() - t_start
        last = rates[-windows:]
        mean = sum(last) / len(last)
        stable = len(last) == windows and mean > 0 and \
            max(abs(r - mean) for r in last) <= tol * mean
        if (el >= a.min_warmup_s and stable) or el >= a.max_warmup_s:
            return el, last


def latency_phase(eng, broker, feeder, bset, parts, rate_img_s, a, ipr):
    """Record-level latency at a fixed offered load (this rank's share ``rate_img_s``): the
    backlog top-up stops, the backlog drains, a native open-loop producer appends the same
    synthetic batches at the offered rate and logs every append (CLOCK_MONOTONIC), the engine
    logs every produce ack on the same clock; the join gives append -> produce-ack per record.
    Returns (latencies_us, achieved images/s, unmatched acks, host dict): the host dict has the
    cgroup's CPU throttling during the window (CFS quota periods in which the rank's cgroup ran
    out of its share: every thread then waits for the next period, a latency tail source)."""
    from gale._native import native
    from gale.metrics import append_to_ack_us, latency_stages_us

    feeder.stop()
    t_end = time.perf_counter() + 10.0
    while time.perf_counter() < t_end:  # drain the backlog phase's records first
        if sum(o["lag"] for o in eng.partition_offsets()) <= 2 * a.batch:
            break
        time.sleep(0.005)
    rf = native().kafka.RateFeeder(broker, "gale-in", parts, bset)
    rf.start(rate_img_s / ipr, feeder._next)
    time.sleep(a.latency_warmup_s)
    broker.take_probes()  # (reset)
    eng.set_ack_log(True)
    c0, t0, cg0, tcp0 = eng.completed, time.perf_counter(), _cgroup_cpu_stat(), _tcp_counters()
    st0 = eng.stats()
    time.sleep(a.latency_s)
    eng.set_ack_log(False)
    st1 = eng.stats()
    dt = time.perf_counter() - t0
    probes = broker.take_probes()
    achieved = (eng.completed - c0) * ipr / dt
    cg1 = _cgroup_cpu_stat()
    host = {}
    if cg0 and cg1:
        d = {k: cg1.get(k, 0) - cg0.get(k, 0) for k in cg1}
        host = {"latency_cg_cores": round(d.get("usage_usec", 0) / 1e6 / dt, 2),
                "latency_cg_throttled_ms": round(d.get("throttled_usec", 0) / 1e3, 1),
                "latency_cg_throttled_periods": int(d.get("nr_throttled", 0)),
                "latency_cg_periods": int(d.get("nr_periods", 0))}
    host["latency_broker_probes"] = probes
    # the GPU ingest's turn per fetch in this window (us): waiting for a lane, host work before
    # the device, the device wait, host work after, and the lane's whole turn
    nf = st1.get("ingest_fetches", 0) - st0.get("ingest_fetches", 0)
    if nf > 0:
        d = {k: (st1.get(k, 0.0) - st0.get(k, 0.0)) / nf * 1e6 for k in (
            "ingest_lane_wait_s", "ingest_prep_s", "ingest_plan_s", "ingest_device_wait_s",
            "ingest_post_s")}
        d["lane_turn"] = (st1["thread_s_ingest"] - st0["thread_s_ingest"]) / nf * 1e6
        host["latency_ingest_us_per_fetch"] = {k.replace("ingest_", "").replace("_s", ""):
                                               round(v, 1) for k, v in d.items()}
        host["latency_ingest_us_per_fetch"]["records"] = round(
            (st1["ingested_records"] - st0["ingested_records"]) / nf, 1)
        # device spans of a sample of the fetches (GALE_INGEST_DEV_TIMING): H2D copies, count
        # pass, parse, and the rest of the same fetches' device wait (queueing behind other
        # streams on the shared hardware queues + completion)
        nd = st1.get("ingest_dev_runs", 0) - st0.get("ingest_dev_runs", 0)
        if nd > 0:
            dv = {k: (st1.get("ingest_dev_" + k + "_s", 0.0) - st0.get("ingest_dev_" + k + "_s", 0.0))
                  / nd * 1e6 for k in ("copy", "count", "parse", "wait")}
            host["latency_ingest_device_us"] = {
                "sampled": int(nd), "copy": round(dv["copy"], 1), "count": round(dv["count"], 1),
                "parse": round(dv["parse"], 1), "host_wait": round(dv["wait"], 1),
                "other": round(dv["wait"] - dv["copy"] - dv["count"] - dv["parse"], 1)}
    tcp1 = _tcp_counters()
    host["latency_tcp"] = {k: tcp1[k] - tcp0.get(k, 0) for k in tcp1 if tcp1[k] != tcp0.get(k, 0)}
    rf.stop()
    ack = eng.take_ack_log()
    app = rf.take_log()
    lat, when = append_to_ack_us(app, ack, with_ack_time=True)
    stages = latency_stages_us(app, ack)
    # per stage: [p50, p99, p999] in ms and the records above 2 ms in that stage alone
    host["latency_stages_ms"] = {
        k: [round(float(np.percentile(v, q)) / 1e3, 3) for q in (50, 99, 99.9)] if len(v) else None
        for k, v in stages.items()}
    host["latency_stage_over_2ms"] = {k: int((v > 2000).sum()) for k, v in stages.items()}
    host["latency_outliers"] = outlier_attribution(stages)
    if a.latency_dump and int(os.environ.get("RANK", "0")) == 0:
        # every 4th record, float32 microseconds (a 2 s window at 1.25 M img/s is 2.5 M records)
        np.savez_compressed(a.latency_dump, latency_us=lat[::4].astype(np.float32),
                            ack_t_ns=when[::4],
                            **{k: v[::4].astype(np.float32) for k, v in stages.items()})
    return lat, achieved, int(len(ack[0]) - len(lat)), host


def outlier_attribution(stages, over_us=2000.0, bucket_ms=10.0):
    """Records whose stage sum (append -> ack) exceeds ``over_us``: how many, which stage held
    the largest share of each (the stage to blame), and how they cluster in time (distinct
    ``bucket_ms`` windows of their fetch time: a few windows = stalls of the whole pipeline, e.g.
    a descheduled thread; many = a diffuse tail)."""
    # (queue = ingest + batching when the log has the split: sum the parts, not both)
    names = [k for k in stages if not (k == "queue" and "ingest" in stages)]
    if not names or not len(stages[names[0]]):
        return {}
    m = np.stack([np.asarray(stages[k], dtype=np.float64) for k in names])
    tot = m.sum(axis=0)
    bad = tot > over_us
    out = {"n": int(bad.sum()), "of": int(len(tot)), "over_us": over_us}
    if bad.any():
        dom = m[:, bad].argmax(axis=0)
        out["dominant_stage"] = {names[i]: int((dom == i).sum()) for i in range(len(names))}
        out["stage_mean_ms"] = {names[i]: round(float(m[i, bad].mean()) / 1e3, 3)
                                for i in range(len(names))}
        # the outliers' positions in the record stream (the stage arrays keep ack-log order,
        # which is time order per sink): spread over the window or bunched?
        pos = np.nonzero(bad)[0]
        out["runs"] = int(1 + (np.diff(pos) > 64).sum())
    return out


def pipeline_path(a, st) -> str:
    """What the timed window actually ran, from the engine's own counters (not the flags)."""
    if a.stub:
        return "kafka-fetch->host-scan->cpu-stub-replica->kafka-produce"
    hops = ["kafka-fetch"]
    recs = max(1.0, st.get("ingested_records", 0))
    pre = st.get("preparsed_records", 0) / recs > 0.5  # the ingest pass parsed the images
    if st.get("ingested_records", 0) > 0:
        hops.append("gpu-ingest(crc32c+count%s%s)" % ("+json-parse" if pre else "",
                                                      ",nibble-link" if a.text_pack else ""))
    else:
        hops.append("host-scan+crc32c")
    batches = max(1.0, st.get("batches", 0))
    step_g = st.get("graph_step_batches", 0) / batches
    fwd_g = st.get("graph_forward_batches", 0) / batches
    if step_g > 0.5:
        hops.append("%s(%sforward%s+status)" %
                    ("hipgraph-step" if a.step_launch == "graph" else "step",
                     "" if pre else "json-parse+", "+format" if a.gpu_encode else ""))
    else:
        hops.append("gpu-json-parse")
        hops.append("hipgraph-forward" if fwd_g > 0.5 else "forward(direct-launch)")
        if a.gpu_encode:
            hops.append("gpu-format")
    hops.append("kafka-produce")
    return "->".join(hops)


def _cpulist(cpus) -> str:
    """Compact CPU list text: {0,1,2,5} -> "0-2,5"."""
    out, run = [], []
    for c in sorted(cpus):
        if run and c == run[-1] + 1:
            run.append(c)
            continue
        if run:
            out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
        run = [c]
    if run:
        out.append(f"{run[0]}-{run[-1]}" if len(run) > 1 else str(run[0]))
    return ",".join(out)


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a, argv) -> int:
    """``bench.py --gpus N`` (N > 1) started as a plain process: this process stays GPU-untouched
    (device_count() only, which initialises no device on this image), starts
    ``torch.distributed.run`` with one rank per GPU as a CHILD process (never an exec), lets rank
    0's JSON line through on the shared stdout and exits with the child's status. Under an
    external torchrun (WORLD_SIZE set) this is skipped and the process is one rank."""
    if not a.stub and not a.shared_gpu_rehearsal:
        import torch

        have = torch.cuda.device_count()
        if a.gpus > have:
            print(f"bench.py: --gpus {a.gpus} but {have} GPU(s) visible (use "
                  "--shared-gpu-rehearsal for a multi-rank rehearsal on fewer GPUs)",
                  file=sys.stderr)
            return 2
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0",
               GALE_BENCH_LAUNCHED="1")
    env.setdefault("OMP_NUM_THREADS", "1")
    p = subprocess.Popen(cmd, cwd=ROOT, env=env)
    try:
        return p.wait()
    except KeyboardInterrupt:
        p.terminate()
        return p.wait()


def size_pipeline(a, cpus: float) -> None:
    """Fill the per-GPU host pipeline sizing left at 0 / -1 from the rank's CPU share."""
    r50 = a.model == "resnet50"
    if a.step_images <= 0:
        # 262144-image steps: ~0.18 s each at 1.5 M img/s (20 steps ~3.6 s), long enough that a
        # single 10-50 ms host hiccup (scheduler, page-cache, neighbour tenants) moves a step's
        # rate by a few percent rather than 10-20 % (131072-image steps: spread 9-20 %,
        # profiles/archive/r3_final_check_session2.jsonl). LeNet-5 runs at ~4 M img/s: its
        # 262144-image steps were 65 ms, shorter than one 100 ms CFS period, and at the cgroup
        # quota they spread by ~100 % (round 4, 3 runs on one box): 4x longer steps
        a.step_images = 4096 if r50 else (1048576 if a.model == "lenet5" else 262144)
    if a.distinct <= 0:
        a.distinct = 256 if r50 else 65536
    if a.batch <= 0:
        # ResNet-50 (BASELINE config 4: dynamic batch <= 256): a 128-image cap halves the
        # latency at the same throughput - the host binds the rate, and a 256-image batch spends
        # ~4 ms filling and ~5.5 ms on the device (profiles/r6_ab_r50_batch.jsonl: 45.2 / 44.7 k
        # img/s, p50 12.3 ms at 256; 46.2 / 42.0 k, p50 6.2 / 6.5 ms at 128; 42.3 / 41.8 k,
        # p50 3.8 ms at 64)
        a.batch = 128 if r50 else 256
    if a.max_wait_us < 0:
        a.max_wait_us = 20000 if r50 else 2000
    big = cpus >= 16
    if a.replicas_per_gpu <= 0:
        if r50:
            a.replicas_per_gpu = 2
        else:
            a.replicas_per_gpu = 6 if big else max(1, min(4, int(cpus // 4)))
    if a.baseline_config == 3:
        a.partitions, a.source_parallelism = 1, 1
    if a.partitions <= 0:
        if r50:
            a.partitions = 12 if big else 4
        else:
            # 11 source threads: with the bounce receive each one packs at ~7 GB/s of text, and
            # fewer threads than 12 contend less at the 16-CPU quota (10: 1.99 vs 1.81 M img/s
            # over 3 interleaved pairs; 9 / 10 / 11: 2.15 / 2.08 / 1.99 M). Below 11 the latency
            # phase, at 0.8 x the higher rate, runs into loopback retransmissions (p99 8-37 ms
            # in some runs against 0.9-1.0 ms with 11; profiles/archive/r4_ab_partitions.jsonl). A larger
            # CPU share per rank (an 8-GPU node without a per-job quota) keeps 12, and so does
            # LeNet-5 (p99 6-112 ms with 10, profiles/archive/r4_ab_lenet_partitions.jsonl)
            a.partitions = (11 if cpus < 24 and a.model != "lenet5" else 12) if big \
                else a.replicas_per_gpu
    if a.decode_threads <= 0:
        # 6 GPU-ingest workers keep more H2D copies in flight on the host link than 4 (higher
        # throughput in 5 of 6 interleaved pairs on two boxes, p50 unchanged; see
        # profiles/archive/r3_decode_threads_ab.txt). With the parse at ingest (round 6) each
        # fetch holds its lane ~30 us longer: 10 lanes keep the ingest stage's p99 at 0.28-0.34 ms
        # against 0.42-0.92 ms with 6 (profiles/r6_ab_ingest_parse.jsonl); a lane mostly sleeps.
        # LeNet-5's fetches carry 4x the records per byte: its lanes queued (lane wait 0.34-0.74
        # ms per fetch in the latency window with 10 against 0.01-0.16 ms with 16,
        # profiles/r6_ingest_breakdown.jsonl). With the 4-wave ResNet-20 forward, 12 lanes
        # beat 10 in 5 of 6 interleaved pairs on two boxes (median 2.24 vs 2.13 M img/s, p50
        # equal; profiles/r6_ab_lanes.jsonl)
        a.decode_threads = ((16 if a.model == "lenet5" else 12) if a.ingest_parse else 6) \
            if big else 2


def print_config(a) -> int:
    """--print-config: the per-rank configuration this command would run at --gpus N (sizing
    from the rank's CPU share, the per-rank CPU slices), without running it."""
    from gale.utils import gpu_numa_node, host_cpus_per_rank, node_cpus, plan_rank_slices

    os.environ.setdefault("LOCAL_WORLD_SIZE", str(1 if a.single_process else a.gpus))
    cpus = host_cpus_per_rank()
    size_pipeline(a, cpus)
    slices = None
    if a.gpus > 1 and a.rank_slices and a.cpus_per_rank == 0 and not a.single_process:
        import torch

        ndev = torch.cuda.device_count()
        if ndev >= a.gpus:
            nodes = [gpu_numa_node(r) for r in range(a.gpus)]
            slices = [_cpulist(x) for x in
                      plan_rank_slices(nodes, {n: node_cpus(n) for n in set(nodes)})]
    print(json.dumps({"n_gpus": a.gpus, "model": a.model, "dtype": a.dtype,
                      "processes": 1 if a.single_process else a.gpus,
                      "host_cpus_per_rank": round(cpus, 2),
                      "replicas_per_gpu": a.replicas_per_gpu,
                      "partitions_per_gpu": a.partitions, "decode_threads": a.decode_threads,
                      "max_batch": a.batch, "max_wait_us": a.max_wait_us,
                      "step_images_per_gpu": a.step_images, "steps": a.steps,
                      "warmup": a.warmup, "rank_cpu_slices": slices}), flush=True)
    return 0


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    a = parse_args(argv)
    if a.print_config:
        return print_config(a)
    if a.gpus > 1 and not a.single_process and "WORLD_SIZE" not in os.environ:
        return launch_ranks(a, argv)
    if a.ingest_dev_timing > 0:
        os.environ.setdefault("GALE_INGEST_DEV_TIMING", str(a.ingest_dev_timing))
    from gale.utils import (cpu_time_split, host_cpus_per_rank, thread_cpu_seconds,
                            thread_ctx_switches)

    # Host pipeline sizing from the rank's CPU share. Throughput is bound by per-connection
    # copy bandwidth and GPU-ingest round trips, not by the total core count: with >= 16 cores
    # per GPU, 12 input partitions (TCP connections), 6 replica streams and 4 ingest workers
    # saturate the share (1.47 M img/s vs 0.97 M with 4/4/2 on one MI355X box,
    # profiles/archive/r2_host_pipeline_shape_ab.txt); smaller shares keep ~4 cores per replica.
    # ResNet-50 records are 1.7 MB of JSON each: the GPU, not the host, sets the pace unless the
    # batches are full, so fewer replicas wait longer for full 256-image batches while 12
    # partitions keep the fetches parallel (29.0 k img/s vs 23.8 k with the CIFAR sizing,
    # profiles/archive/r2_configs_1_4_e2e.txt)
    size_pipeline(a, host_cpus_per_rank())
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # GPUs driven by this process (> 1 only in --single-process mode)
    local_gpus = a.gpus if a.single_process else 1
    if a.single_process and world > 1:
        raise SystemExit("bench.py: --single-process runs as ONE process (no torchrun)")
    if world > 1 and world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started {world} ranks")
    import torch
    import torch.distributed as dist

    use_gpu = not a.stub
    if use_gpu and not torch.cuda.is_available():
        raise SystemExit("bench.py: no GPU visible (use --stub for the CPU plumbing run)")
    if use_gpu and local_gpus > torch.cuda.device_count():
        raise SystemExit(f"bench.py: {local_gpus} GPUs requested, "
                         f"{torch.cuda.device_count()} visible")
    rank_index = local_rank  # (the rank's index on this node, also in the rehearsal)
    if use_gpu and a.shared_gpu_rehearsal:
        local_rank %= torch.cuda.device_count()
    pinned_cpus = set()
    if use_gpu:
        torch.cuda.set_device(local_rank)
        if a.numa_pin and local_gpus == 1:
            from gale.utils import (cgroup_cpu_quota, gpu_numa_node, node_cpus, pin_cpus,
                                    pin_to_gpu_numa, plan_rank_slices)

            local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
            if a.cpus_per_rank < 0:
                q = cgroup_cpu_quota()
                a.cpus_per_rank = int(q // max(1, local_world)) if q else 0
            if a.cpus_per_rank == 0 and local_world > 1 and a.rank_slices:
                # disjoint per-rank slices of each GPU's NUMA node (profiles/r5_slices_ab.jsonl,
                # profiles/r5_host_budget.txt); the rehearsal's ranks share GPU 0's node
                ndev = torch.cuda.device_count()
                nodes = [gpu_numa_node(r % ndev if a.shared_gpu_rehearsal else r)
                         for r in range(local_world)]
                plan = plan_rank_slices(nodes, {n: node_cpus(n) for n in set(nodes)})
                pinned_cpus = pin_cpus(plan[rank_index])
            else:
                pinned_cpus = pin_to_gpu_numa(local_rank, a.cpus_per_rank, smt=a.slice_smt)
    if world > 1:
        from gale.parallel.group import init_rank_group

        init_rank_group(local_rank, use_gpu, shared_gpu=a.shared_gpu_rehearsal)

    from gale._native import native
    from gale.config import GaleConfig
    from gale.data import synthetic_images
    from gale.engine import Engine
    from gale.models import get_model

    net = get_model(a.model)
    native().set_pack_stream_stores(a.pack_nt)
    K = native().kafka
    ipr = a.images_per_record
    parts_per_rank = a.partitions * local_gpus
    # records per RecordBatch: a producer's batch (rate mode: small batches, arrivals are not
    # bursty; the feeder keeps to ~10k appends/s) ...
    rpb = min(64, max(8, int(a.rate // 10000))) if a.rate > 0 else 64
    # ... and at most ~4 MB per RecordBatch, as a producer's batch.size would keep it: a fetch
    # always returns at least one whole batch (KIP-74), so 64 ResNet-50 records (1.7 MB each)
    # in one batch would turn every fetch into a 109 MB response
    rec_bytes = 12 * int(np.prod(net.input_shape)) * ipr  # ~Java float text per record
    rpb = max(1, min(rpb, (4 << 20) // rec_bytes))
    distinct = max(rpb * ipr, (a.distinct // (rpb * ipr)) * rpb * ipr)
    t_enc = time.perf_counter()
    imgs = synthetic_images(distinct, net.input_shape, seed=1234 + rank)
    enc_threads = a.encode_threads or max(1, int(host_cpus_per_rank()))
    bset = K.synthetic_batches(imgs, ipr, rpb, enc_threads)
    # the latency phase's producer batches (--latency-batch-records; 0 = the same batches as the
    # backlog): smaller batches make arrivals less bursty, as a kafka-clients producer with its
    # 16 KB batch.size sends one ~35 KB record per batch
    lat_bset = bset
    lrpb = min(a.latency_batch_records, rpb) if a.latency_batch_records > 0 else rpb
    if lrpb != rpb:
        lat_bset = K.synthetic_batches(imgs[:max(lrpb * ipr, len(imgs) // 4)], ipr, lrpb,
                                       enc_threads)
    del imgs
    t_enc = time.perf_counter() - t_enc

    # byte retention per partition: far above the backlog the feeder keeps ahead of the
    # consumers (input batches are shared references, so input retention costs no copies), but
    # bounded, so the output topic (~0.3 GB/s of predictions at 1.5 M img/s) does not grow the
    # broker's memory for the whole run
    broker = K.Broker(node_id=rank, max_message_bytes=256 << 20, retention_bytes=2 << 30,
                      zero_copy=a.broker_zero_copy, log_append_time=True)
    broker.start()
    n_parts = world * parts_per_rank
    if world > 1:
        ports = [None] * world
        dist.all_gather_object(ports, broker.port)
        broker.set_cluster([(r, "127.0.0.1", int(ports[r])) for r in range(world)])
    broker.create_topic("gale-in", n_parts)
    broker.create_topic("gale-out", world)
    my_parts = [p for p in range(n_parts) if p % world == rank]  # the partitions this rank leads
    step_images = a.step_images * local_gpus  # (a step is per GPU)
    step_records = -(-step_images // ipr)
    feeder = Feeder(broker, "gale-in", my_parts, bset, rate=a.rate,
                    ahead_records=-(-max(step_records, 65536 // ipr) // len(my_parts)))
    if a.rate <= 0:
        feeder.fill(feeder.ahead)
    if world > 1:
        dist.barrier()  # every broker of the cluster is up and has its topics

    cfg = GaleConfig(topology_name=f"bench-r{rank}", input_topic="gale-in",
                     output_topic="gale-out", bootstrap=f"127.0.0.1:{broker.port}",
                     partitions=",".join(map(str, my_parts)),
                     group_id="bench", start_offset="earliest", model=a.model, dtype=a.dtype,
                     max_batch=a.batch, max_wait_us=a.max_wait_us,
                     queue_depth=max(1, a.queue_batches * a.batch // ipr),
                     source_parallelism=a.source_parallelism or len(my_parts),
                     sink_parallelism=a.sink_parallelism * local_gpus,
                     replicas=a.replicas_per_gpu * local_gpus,
                     decode_threads=a.decode_threads, slo_p99_ms=a.slo_p99_ms,
                     gpu_wait_poll_us=a.gpu_wait_poll_us, gpu_ingest=a.gpu_ingest, gpu_encode=a.gpu_encode,
                     replica_priority=a.replica_priority, step_launch=a.step_launch,
                     text_pack=a.text_pack, text_pack_bounce=a.text_pack_bounce,
                     ingest_parse=a.ingest_parse, partition_max_kb=a.partition_max_kb,
                     text_pack_window_kb=a.text_pack_window_kb,
                     pinned_fetch_mb=a.pinned_fetch_mb,
                     stub=a.stub, stub_null=a.stub_null, commit_interval_ms=500,
                     check_crcs=a.check_crcs,
                     output_partition=rank if a.local_output and world > 1 else -1,
                     producer_buffer_mb=a.producer_buffer_mb,
                     locality_split=a.locality_split, fetch_min_bytes=a.fetch_min_bytes,
                     fetch_max_wait_ms=a.fetch_max_wait_ms, recv_lowat_kb=a.recv_lowat_kb,
                     use_graph=a.graph, graph_step=a.graph_step,
                     producer_request_kb=a.producer_request_kb)
    devices = (list(range(local_gpus)) if local_gpus > 1 else [local_rank]) if use_gpu else None
    # ONE engine: warm-up and timed window are the same steady-state pipeline (connections,
    # pinned fetch buffers, captured graphs all warm); the timed window starts at a barrier
    # once every rank has warmed up and ends when K more steps completed on this rank.
    # weights: seeded on rank 0 (or the first GPU), RCCL-broadcast to every other GPU
    eng = Engine(cfg, devices=devices,
                 stub_localities=tuple(range(local_gpus)) if a.stub and local_gpus > 1 else ())
    eng.start()
    feeder.start(eng)
    timeline = Timeline(a.timeline, a.timeline_ms, broker) if a.timeline and rank == 0 else None
    if timeline:
        timeline.start(eng)
    warm_s, warm_rates = warm_up(eng, max(1, a.warmup) * step_records, a)
    if timeline:
        timeline.phase = "timed"
    warm_done = eng.completed
    if world > 1:
        dist.barrier()
    if use_gpu:
        torch.cuda.synchronize()
    eng.reset_stats()
    cpu0 = thread_cpu_seconds()
    ctx0, split0 = thread_ctx_switches(), cpu_time_split(pinned_cpus)
    cgt0 = _cgroup_cpu_stat()
    c0 = eng.completed
    t0 = time.perf_counter()
    m0 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
    marks = []  # (s since t0, records completed): step boundaries for the per-step rates
    reached = True
    for k in range(1, a.steps + 1):
        if not eng.wait_completed(c0 + k * step_records, a.timeout):
            reached = False
            break
        # the completing thread's own clock reading of the crossing: this thread's wake-up runs
        # late by a varying few ms on a saturated host, and a late mark shortens the next step
        # (an alternating fast / slow pattern that is the measurement, not the pipeline)
        ns, c = eng.last_wait()
        if ns > 0:
            marks.append(((ns - m0) * 1e-9, c))
        else:
            marks.append((time.perf_counter() - t0, eng.completed))
    if use_gpu:
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    cpu1 = thread_cpu_seconds()
    ctx1, split1 = thread_ctx_switches(), cpu_time_split(pinned_cpus)
    cgt1 = _cgroup_cpu_stat()
    # cgroup CPU accounting of the timed window: at the CPU quota the CFS bandwidth controller
    # stops the whole group for the rest of each 100 ms period, which alternates fast and slow
    # steps (the step spread) without changing the mean
    cg_timed = {}
    if cgt0 and cgt1:
        d = {k: cgt1.get(k, 0) - cgt0.get(k, 0) for k in cgt1}
        cg_timed = {"cores": round(d.get("usage_usec", 0) / 1e6 / max(elapsed, 1e-9), 2),
                    "throttled_ms": round(d.get("throttled_usec", 0) / 1e3, 1),
                    "throttled_periods": int(d.get("nr_throttled", 0)),
                    "periods": int(d.get("nr_periods", 0))}
    done_records = eng.completed - c0
    st = eng.stats()
    if timeline:
        timeline.phase = "latency"
    if not reached:
        raise SystemExit(f"rank {rank}: timed out after {elapsed:.1f}s "
                         f"({done_records}/{a.steps * step_records} records)")
    images = done_records * ipr  # >= K steps (completions arrive a micro-batch at a time)
    t = torch.tensor([elapsed, float(images)], dtype=torch.float64)
    if world > 1:
        tt = t.cuda() if use_gpu and not a.shared_gpu_rehearsal else t
        mx = tt.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = tt.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed_max, total_images = float(mx[0]), float(sm[1])
        # every rank's own view, for the JSON line: its partitions, output partition, window,
        # images, host slice and busy cores (imbalance between ranks shows up here)
        mine = {"rank": rank, "partitions": my_parts, "output_partition": cfg.output_partition,
                "timed_s": round(elapsed, 6), "images": int(images),
                "img_s": round(images / max(elapsed, 1e-9), 1),
                "cpus": _cpulist(pinned_cpus),
                "cores": round(sum(cpu1[k] - cpu0[k] for k in cpu1) / max(elapsed, 1e-9), 2)}
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    else:
        elapsed_max, total_images = elapsed, float(images)
        per_rank = None
    value = total_images / elapsed_max
    n_gpus = world * local_gpus
    lat_us, lat_achieved, lat_unmatched, lat_host = None, 0.0, 0, {}
    offered = a.latency_load * value  # whole job, images/s

    def measure(load_img_s):
        if world > 1:
            dist.barrier()
        lu, ach, unm, hst = latency_phase(eng, broker, feeder, lat_bset, my_parts,
                                          load_img_s / world, a, ipr)
        if world > 1:
            # every rank's samples (subsampled to <= 200k) and achieved rate to rank 0
            if len(lu) > 200_000:
                lu = lu[np.random.default_rng(rank).choice(len(lu), 200_000, replace=False)]
            got = [None] * world
            dist.all_gather_object(got, (lu, ach, unm))
            lu = np.concatenate([g[0] for g in got])
            ach = sum(g[1] for g in got)
            unm = sum(g[2] for g in got)
        return lu, ach, unm, hst

    sweep = []
    if a.latency_load > 0 and a.rate <= 0:
        lat_us, lat_achieved, lat_unmatched, lat_host = measure(offered)
        for frac in [float(x) for x in a.latency_sweep.split(",") if x.strip()]:
            for _ in range(max(1, a.latency_repeat)):
                lu, ach, unm, hst = measure(frac * value)
                if len(lu):
                    sweep.append({"load": frac, "offered_img_s": round(frac * value, 1),
                                  "achieved_img_s": round(ach, 1),
                                  "p50_ms": round(float(np.percentile(lu, 50)) / 1e3, 3),
                                  "p99_ms": round(float(np.percentile(lu, 99)) / 1e3, 3),
                                  "p999_ms": round(float(np.percentile(lu, 99.9)) / 1e3, 3),
                                  "samples": int(len(lu)), "unmatched": unm,
                                  "stages_ms": hst.get("latency_stages_ms"),
                                  "cg_throttled_ms": hst.get("latency_cg_throttled_ms"),
                                  "broker_probes": hst.get("latency_broker_probes"),
                                  "tcp": hst.get("latency_tcp")})
    if timeline:
        timeline.stop()
    if world > 1:
        dist.barrier()
    feeder.stop()
    eng.stop()
    if world > 1:
        dist.barrier()  # (sinks produce to every rank's broker: stop brokers after all engines)
    broker.stop()
    if rank == 0 and elapsed_max < 1.0:
        print(f"bench.py: timed window {elapsed_max:.3f} s < 1 s: raise --step-images",
              file=sys.stderr)
    if rank == 0:
        # per-step rates from (time, completed) marks; a completion burst can cross several step
        # boundaries at once, so intervals shorter than half a mean step are merged with the next
        step_rates, ta, ca = [], 0.0, c0
        for tb, cb in marks:
            if tb - ta >= 0.5 * elapsed / max(1, len(marks)) and cb > ca:
                step_rates.append((cb - ca) * ipr / (tb - ta))
                ta, ca = tb, cb
        step_rates = step_rates or [value]
        med = statistics.median(step_rates)
        cores = {k: round((cpu1[k] - cpu0[k]) / elapsed, 2) for k in cpu1}
        out = {
            "metric": METRICS[a.model], "value": round(value, 1), "unit": "images/s",
            "n_gpus": n_gpus,
            "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed_max / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
            "data": f"synthetic ({distinct} distinct uniform [0,1) "
                    f"{'x'.join(map(str, net.input_shape))} images as InstObj JSON records, "
                    "Java float format, fed through an embedded Kafka-protocol broker cluster, "
                    "one broker per rank); random-init weights (seed 0) RCCL-broadcast from "
                    "rank 0",
            "step": f"{a.step_images} images per GPU through fetch->parse->forward->produce-ack",
            "config": {"model": a.model,
                       # images per timed step over the whole job (the unit ms_per_step times);
                       # each forward launch runs a micro-batch of <= max_batch images
                       "global_batch": a.step_images * n_gpus,
                       "seq_len": None, "parallelism": f"dp{n_gpus}",
                       "processes": world,
                       "launcher": ("torch.distributed.run child of bench.py"
                                    if os.environ.get("GALE_BENCH_LAUNCHED") else
                                    "torch.distributed.run" if world > 1 else
                                    "single process"),
                       "images_per_record": ipr, "max_batch": a.batch,
                       "max_wait_us": a.max_wait_us, "replicas_per_gpu": a.replicas_per_gpu,
                       "decode_threads": a.decode_threads,
                       "locality_split": a.locality_split,
                       "partitions": n_parts,
                       "source_threads_per_gpu": a.source_parallelism or a.partitions,
                       "baseline_config": a.baseline_config or None,
                       "step_images_per_gpu": a.step_images,
                       "path": pipeline_path(a, st)},
            "load": (f"offered {a.rate:.0f} images/s per GPU" if a.rate > 0
                     else "value: backlog kept ahead of the consumers (max throughput); "
                          "latency: a second phase at a fixed offered load"),
            "timed_s": round(elapsed_max, 3),
        }
        if per_rank:
            out["ranks"] = per_rank
        if lat_us is not None and len(lat_us):
            out.update({
                "p50_latency_ms": round(float(np.percentile(lat_us, 50)) / 1e3, 3),
                "p99_latency_ms": round(float(np.percentile(lat_us, 99)) / 1e3, 3),
                "latency_definition": "Kafka record append -> prediction produce-ack, per "
                                      "record, CLOCK_MONOTONIC (us resolution), at a fixed "
                                      "offered load (open-loop native producer)",
                "latency_offered_img_s": round(offered, 1),
                "latency_achieved_img_s": round(lat_achieved, 1),
                "latency_samples": int(len(lat_us)),
                "latency_unmatched": lat_unmatched,
                "p90_latency_ms": round(float(np.percentile(lat_us, 90)) / 1e3, 3),
                "p999_latency_ms": round(float(np.percentile(lat_us, 99.9)) / 1e3, 3),
                **lat_host,  # rank 0's cgroup during the latency window
            })
            if sweep:
                out["latency_sweep"] = sweep
        else:
            out.update({
                "p50_latency_ms": round(st["e2e_us_p50"] / 1e3, 3),
                "p99_latency_ms": round(st["e2e_us_p99"] / 1e3, 3),
                "latency_definition": "fetch -> produce-ack under the backlog (includes "
                                      "queueing; no offered-load phase)",
            })
        out.update({
            "backlog_fetch_to_ack_ms_p50": round(st["e2e_us_p50"] / 1e3, 3),
            "backlog_fetch_to_ack_ms_p99": round(st["e2e_us_p99"] / 1e3, 3),
            "backlog_record_e2e_ms_p50": round(st["record_e2e_ms_p50"], 2),
            "backlog_record_e2e_ms_p99": round(st["record_e2e_ms_p99"], 2),
            "device_ms_p50": round(st["device_us_p50"] / 1e3, 3),
            "batch_images_mean": round(st["batch_images_mean"], 1),
            "step_rate_spread": {"min": round(min(step_rates)), "median": round(med),
                                 "max": round(max(step_rates)),
                                 "range_pct": round(100 * (max(step_rates) - min(step_rates))
                                                    / med, 1)},
            "step_rates": [round(r) for r in step_rates],
            "timed_cgroup_rank0": cg_timed,
            "warmup_s": round(warm_s, 2), "warmup_rates": [round(r) for r in warm_rates],
            "json_mb_per_s_rank0": round(st["bytes_in"] / elapsed / 1e6, 1),
            # host -> GPU link bytes per fetched text byte (nibble transport: ~0.5)
            "link_ratio_rank0": round(st["ingest_link_bytes"] / st["ingest_text_bytes"], 4)
            if st.get("ingest_text_bytes") else None,
            "cpu_cores_busy_rank0": round(sum(cores.values()), 2),
            "cpu_cores_by_stage_rank0": cores,
            "encode_s": round(t_enc, 1),
            "cpus_pinned_rank0": len(pinned_cpus),
            "cpu_slice_rank0": _cpulist(pinned_cpus),
            # per stage, thousands of context switches per second: [voluntary, involuntary]
            "ctx_k_per_s_rank0": {k: [round((ctx1[k][0] - ctx0[k][0]) / elapsed / 1e3, 1),
                                      round((ctx1[k][1] - ctx0[k][1]) / elapsed / 1e3, 1)]
                                  for k in ctx1 if k in ctx0},
            # the pinned CPUs' time by /proc/stat category (whole machine when unpinned), in
            # cores: softirq is the loopback receive processing, charged to no thread
            "slice_cores_rank0": {k: round((split1[k] - split0.get(k, 0.0)) / elapsed, 2)
                                  for k in ("user", "system", "softirq", "irq", "idle")
                                  if k in split1},
            "steals": int(st.get("steals", 0)),
            "warmup_records": warm_done,
        })
        if a.all_stats:
            out["engine_stats_rank0"] = {k: round(v, 3) for k, v in st.items()}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
