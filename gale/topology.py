"""Topology lifecycle: submit / run for a duration / kill / list (R2, E4, X5).

The reference submits its DAG to Nimbus over Thrift (``StormSubmitter.submitTopology``,
MainTopology.java:69), blocks the client for one hour (:71) and then kills the topology with
``KillOptions(wait_secs=0)`` (:73-77); Thrift errors go to a log/print ladder
(AlreadyAlive / InvalidTopology / Authorization / NotAlive, :79-91). gale has no cluster
manager to talk to: a topology is a local process (or one process per GPU under
``torch.distributed.run``) and a lockfile/pidfile registry keyed by topology name provides the
same lifecycle semantics:

* ``Registry.register`` refuses a name held by a live process -> ``AlreadyAliveError``;
* ``Registry.kill(name, wait_secs)`` sends SIGTERM (graceful drain: sources stop, queued
  records finish, the sink is flushed, offsets committed) and SIGKILL after ``wait_secs``
  (``wait_secs=0`` is the reference's immediate kill) -> ``NotAliveError`` if not running;
* ``run_topology`` serves until ``duration`` elapses (reference: 3600 s) or a signal arrives.
"""

from __future__ import annotations

import fcntl
import json
import logging
import os
import signal
import socket
import threading
import time
from typing import Dict, List, Optional

from gale.config import GaleConfig

log = logging.getLogger("gale.topology")


class TopologyError(RuntimeError):
    pass


class AlreadyAliveError(TopologyError):
    pass


class NotAliveError(TopologyError):
    pass


class InvalidTopologyError(TopologyError):
    pass


class RankFailedError(TopologyError):
    """Every replica of this rank is dead (e.g. a hung device the watchdog gave up on), or an
    output could not be delivered under at-least-once delivery: the process exits non-zero so
    the rank supervisor (--ranks) replaces it, resuming from the committed offsets."""


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


class Registry:
    """Directory of ``<name>.json`` records, each guarded by an flock held by the owner."""

    def __init__(self, root: str):
        self.root = root
        os.makedirs(root, exist_ok=True)
        self._held: Dict[str, int] = {}

    def _path(self, name: str) -> str:
        if not name or "/" in name or name.startswith("."):
            raise InvalidTopologyError(f"invalid topology name {name!r}")
        return os.path.join(self.root, name + ".json")

    def register(self, name: str, info: dict) -> None:
        path = self._path(name)
        fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o644)
        try:
            fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
        except BlockingIOError:
            os.close(fd)
            raise AlreadyAliveError(f"Topology {name} is already alive") from None
        rec = dict(info, name=name, pid=os.getpid(), host=socket.gethostname(),
                   started=time.time())
        os.ftruncate(fd, 0)
        os.write(fd, json.dumps(rec).encode())
        os.fsync(fd)
        self._held[name] = fd

    def unregister(self, name: str) -> None:
        fd = self._held.pop(name, None)
        if fd is None:
            return
        try:
            os.unlink(self._path(name))
        except FileNotFoundError:
            pass
        fcntl.flock(fd, fcntl.LOCK_UN)
        os.close(fd)

    def get(self, name: str) -> Optional[dict]:
        try:
            with open(self._path(name)) as fh:
                rec = json.load(fh)
        except (FileNotFoundError, json.JSONDecodeError):
            return None
        return rec if _alive(int(rec.get("pid", -1))) else None

    def list(self) -> List[dict]:
        out = []
        for fn in sorted(os.listdir(self.root)):
            if fn.endswith(".json"):
                rec = self.get(fn[:-5])
                if rec:
                    out.append(rec)
        return out

    def kill(self, name: str, wait_secs: float = 0.0) -> None:
        rec = self.get(name)
        if rec is None:
            raise NotAliveError(f"Topology {name} is not alive")
        pid = int(rec["pid"])
        os.kill(pid, signal.SIGTERM)
        deadline = time.time() + max(0.0, wait_secs)
        while time.time() < deadline and _alive(pid):
            time.sleep(0.05)
        if wait_secs > 0 and _alive(pid):
            os.kill(pid, signal.SIGKILL)


def _dist_env():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _pin_single_gpu(cfg: GaleConfig, devices) -> None:
    """One GPU per process (a rank, or a single-GPU box): keep the host pipeline on its NUMA
    node. A process spreading replicas over several GPUs is left unpinned."""
    import torch

    if devices is None:
        n = torch.cuda.device_count() if torch.cuda.is_available() else 0
        devices = [0] if (n == 1 or cfg.gpus == 1) else []
    if len(devices) == 1:
        from gale.utils import pin_to_gpu_numa

        cpus = pin_to_gpu_numa(devices[0])
        if cpus:
            log.info("host pipeline pinned to the %d CPUs of GPU %d's NUMA node", len(cpus),
                     devices[0])


def run_topology(cfg: GaleConfig, stop_event: Optional[threading.Event] = None,
                 install_signals: bool = True) -> dict:
    """Serve ``cfg`` until its duration elapses, a signal arrives or ``stop_event`` is set.
    Returns the final engine stats."""
    from gale.engine import Engine
    from gale.metrics import MetricsServer, Reporter

    rank, world, local_rank = _dist_env()
    supervised = bool(os.environ.get("GALE_SUPERVISED"))
    # a supervised rank registers as NAME.r<rank> even alone (--ranks 1): the supervisor holds NAME
    name = cfg.topology_name if world == 1 and not supervised else f"{cfg.topology_name}.r{rank}"
    registry = Registry(cfg.registry_dir)
    registry.register(name, {"input_topic": cfg.input_topic, "output_topic": cfg.output_topic,
                             "bootstrap": cfg.bootstrap, "model": cfg.model, "rank": rank})
    broker = None
    engine = None
    stop_event = stop_event or threading.Event()
    old_handlers = {}
    try:
        if cfg.embedded_broker and rank == 0:
            broker = start_embedded_broker(cfg)
        devices = None
        incarnation = int(os.environ.get("GALE_RANK_INCARNATION", "0"))
        if incarnation > 0 and cfg.start_offset != "committed":
            # a respawned rank resumes where its predecessor's commits end (storm-kafka: a
            # restarted worker of the same topology reads its ZK offsets; ignoreZkOffsets only
            # applies to a new submission); "latest" would skip whatever was in flight
            if cfg.start_offset == "earliest":
                cfg.auto_offset_reset = "earliest"
            cfg.start_offset = "committed"
        if world > 1 and not cfg.stub:
            dev = local_rank
            if cfg.shared_gpu_rehearsal:
                import torch

                dev = local_rank % max(1, torch.cuda.device_count())
            devices = [dev]
            if incarnation == 0:
                from gale.parallel.group import init_rank_group

                init_rank_group(dev, use_gpu=True, shared_gpu=cfg.shared_gpu_rehearsal)
            # a respawned rank (incarnation > 0) has no group to join: it materialises the
            # weights itself from the same seed / --weights file (Storm's prepare() reload)
        if world > 1 and not cfg.partitions and not cfg.group_membership:
            cfg.partitions = rank_partitions(cfg, rank, world)
        if cfg.numa_pin and not cfg.stub:
            _pin_single_gpu(cfg, devices)
        engine = Engine(cfg, devices=devices)
        if supervised and world > 1:
            # the group existed for the one-time weight broadcast: a supervised rank may die and
            # be respawned later, so no rank keeps a communicator with a peer that can vanish
            import torch.distributed as dist

            if dist.is_initialized():
                dist.destroy_process_group()
        if install_signals and threading.current_thread() is threading.main_thread():
            for sig in (signal.SIGTERM, signal.SIGINT):
                old_handlers[sig] = signal.signal(sig, lambda *_: stop_event.set())
        engine.start()
        log.info("topology %s running: %s -> %s on %s (model %s, %d replica(s))", name,
                 cfg.input_topic, cfg.output_topic, cfg.bootstrap, cfg.model,
                 len(engine.replica_stats()))
        ready = os.environ.get("GALE_READY_FILE")
        if ready:  # the supervisor's start-up barrier
            with open(ready + ".tmp", "w") as fh:
                json.dump({"rank": rank, "pid": os.getpid(), "incarnation": incarnation}, fh)
            os.replace(ready + ".tmp", ready)
        labels = {"topology": name, "rank": rank}
        if supervised:
            labels["rank_restarts"] = incarnation
        reporter = Reporter(engine.stats, cfg.metrics_interval, path=cfg.metrics_file,
                            labels=labels,
                            extra_fn=lambda: {"partitions": sorted(
                                o["partition"] for o in engine.partition_offsets())}).start()
        http = None
        if cfg.metrics_port >= 0:
            port = cfg.metrics_port + local_rank if cfg.metrics_port > 0 else 0
            http = MetricsServer(engine, port, labels=labels).start()
            log.info("metrics: http://127.0.0.1:%d/metrics (Prometheus), /stats (JSON)",
                     http.port)
        failed = _serve_until_done(engine, cfg, stop_event)
        if http is not None:
            http.stop()
        reporter.stop(final=False, close=False)
        engine.stop()
        final = reporter.report()
        reporter.close()
        if failed:
            raise RankFailedError(f"rank {rank}: {failed}")
        return dict(engine.stats(), final=final)
    finally:
        if engine is not None and engine.running:
            engine.stop()
        if broker is not None:
            broker.stop()
        for sig, h in old_handlers.items():
            signal.signal(sig, h)
        registry.unregister(name)


def _serve_until_done(engine, cfg: GaleConfig, stop_event: threading.Event) -> str:
    """Serve until the duration elapses or ``stop_event`` is set; returns "" then, or why the
    rank can no longer serve: no replica alive for longer than a replica restart could take
    (the watchdog killed them on a hung device, or they failed past --max-restarts)."""
    deadline = time.monotonic() + cfg.duration if cfg.duration > 0 else None
    grace = max(2.0, 2 * cfg.restart_backoff_ms / 1e3 + 1.0)
    dead_since = None
    while True:
        wait = 0.25 if deadline is None else min(0.25, max(0.0, deadline - time.monotonic()))
        if stop_event.wait(wait) or (deadline is not None and time.monotonic() >= deadline):
            return ""
        st = engine.stats()
        if st.get("delivery_failed", 0):
            return (f"at-least-once delivery failed: {int(st.get('undelivered', 0))} output(s) "
                    f"not acknowledged after {cfg.producer_retries} retries; offsets stay "
                    f"uncommitted from the first of them")
        alive = st.get("replicas_alive", 1)
        if alive > 0:
            dead_since = None
            continue
        now = time.monotonic()
        dead_since = dead_since or now
        if now - dead_since >= grace:
            return f"every replica is dead (replicas_alive 0 for {now - dead_since:.1f} s)"


def rank_partitions(cfg: GaleConfig, rank: int, world: int) -> str:
    """One process per GPU: rank r consumes the partitions p with p % world == r (P2)."""
    from gale._native import native

    c = native().kafka.Consumer(cfg.bootstrap)
    c.assign(cfg.input_topic, [])
    parts = [p for p in c.assignment() if p % world == rank]
    if not parts:
        raise InvalidTopologyError(f"rank {rank}: no partitions of {cfg.input_topic} "
                                   f"(world {world}); create at least {world} partitions")
    return ",".join(str(p) for p in parts)


def start_embedded_broker(cfg: GaleConfig):
    """In-process Kafka-protocol broker on the bootstrap address (first host:port)."""
    from gale._native import native

    first = cfg.bootstrap.split(",")[0].strip()
    host, _, port = first.rpartition(":")
    b = native().kafka.Broker(host=host or "127.0.0.1", port=int(port or 9092),
                              default_partitions=cfg.broker_partitions,
                              max_message_bytes=256 << 20)
    b.start()
    for t in (cfg.input_topic, cfg.output_topic):
        b.create_topic(t, cfg.broker_partitions)
    log.info("embedded broker on %s:%d (%d partition(s) per topic)", host, b.port,
             cfg.broker_partitions)
    return b
