"""One configuration object for a gale topology.

The reference spreads its configuration over three layers: compiled-in constants
(``NUM_WORKERS=8, KAFKA_SPOUT_PARAL=2, INFERENCE_BOLT_PARAL=4, KAFKA_BOLT_PARAL=2``,
MainTopology.java:25-28), hard-coded ``zkHosts`` / ``bootstrap`` strings that must be edited in
source (:33-34, README.md:38) and three positional CLI args (:36-38). gale keeps the positional
``<TOPOLOGY_NAME> <INPUT_TOPIC> <OUTPUT_TOPIC>`` contract and turns every knob into a field with
precedence

    CLI flag  >  environment (GALE_<FIELD>)  >  TOML file (--config)  >  default.
"""

from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field, fields
from typing import Any, Dict, List, Optional

CHOICES = {
    "replica_priority": ("normal", "high"),
    "step_launch": ("graph", "direct"),
    "sink_mode": ("async", "sync", "fire-and-forget"),
    "start_offset": ("latest", "earliest", "committed"),
    "auto_offset_reset": ("latest", "earliest"),
    "delivery": ("auto", "at-most-once", "at-least-once"),
    "value_format": ("json", "json-string"),
    "on_error": ("null", "error-json", "drop"),
    "output_key": ("none", "input"),
    "float_format": ("jdk19", "java8"),
    "assignor": ("range", "roundrobin", "load-aware"),
    "compression": ("none", "gzip", "snappy", "lz4", "zstd"),
    # compute dtype of the GPU kernels (MFMA bf16 / OCP e4m3 fp8 serving plans; fp32 = the
    # reference-precision plan on the fp32 matrix core, every tensor binary32 like the
    # reference's TF graph, InferenceBolt.java:80-86); inputs and the softmax output are fp32
    "dtype": ("bf16", "fp8", "fp32"),
    "model": ("lenet5", "resnet20", "resnet50"),
}


@dataclass
class GaleConfig:
    # positional contract (MainTopology.java:36-38)
    topology_name: str = "gale"
    input_topic: str = ""
    output_topic: str = ""
    # Kafka (R4, R5; the reference's zkHosts/bootstrap strings, MainTopology.java:33-34)
    bootstrap: str = "127.0.0.1:9092"
    embedded_broker: bool = False      # run an in-process broker on the bootstrap address
    broker_partitions: int = 1         # partitions of auto-created topics (embedded broker)
    group_id: str = ""                 # default: the topology name
    partitions: str = ""               # comma-separated input partitions (empty = all)
    start_offset: str = "latest"       # reference: LatestTime + ignoreZkOffsets (:101-102)
    auto_offset_reset: str = "latest"  # start_offset=committed / group-managed partitions with no
                                       # committed offset start here (Kafka auto.offset.reset)
    commit_interval_ms: int = 2000
    fetch_min_bytes: int = 1           # Kafka fetch.min.bytes of the consumers (long-poll size)
    fetch_max_wait_ms: int = 20        # Kafka fetch.max.wait.ms
    recv_lowat_kb: int = -1            # consumers wake per this many KB of a large fetch
                                       # response (SO_RCVLOWAT per receive call); 0 = per segment,
                                       # -1 = the bounce window with the bounce receive, else 0
    fetch_max_kb: int = 16384          # Kafka fetch.max.bytes (per fetch response)
    partition_max_kb: int = 8192       # Kafka max.partition.fetch.bytes
    pinned_fetch_mb: int = 4096        # pinned fetch-buffer budget per GPU (x2 with text_pack);
                                       # when it is spent the sources wait for a free buffer
    # elastic data parallelism: every process of the group shares the input partitions through
    # Kafka consumer-group membership; dead members' partitions move to the survivors
    group_membership: bool = False
    session_timeout_ms: int = 6000
    rebalance_timeout_ms: int = 8000
    heartbeat_interval_ms: int = 500
    assignor: str = "range"            # range | roundrobin | load-aware (capacity-weighted,
                                       # sticky; a member lagging behind triggers a rebalance)
    lag_rebalance_records: int = 0     # load-aware trigger: own lag above this and growing for
                                       # 1 s (0 = 8 x max_batch x replicas)
    rebalance_cooldown_ms: int = 10000  # load-aware: at most one lag-triggered rebalance per
                                        # cooldown
    decode_threads: int = 2            # CRC32C + envelope-scan workers behind each consumer
    check_crcs: bool = True            # Kafka consumer check.crcs
    gpu_ingest: bool = True            # CRC32C + image counts of pinned fetch buffers on the GPU
                                       # (the host reads only Kafka framing; csrc/runtime/ingest.h)
    text_pack: bool = True             # GPU ingest: sources nibble-pack fetch bodies for the
                                       # PCIe link, expanded on the device (text_pack.h); needs
                                       # AVX-512 VBMI; for hosts with idle cores behind a
                                       # link-bound GPU (profiles/archive/r3_nibble_transport_ab.txt)
    text_pack_bounce: bool = True      # with text_pack: fetch bodies go through a cache-resident
                                       # window; the pinned chunk gets the packed text and a
                                       # sparse framing copy only (csrc/runtime/pack_tap.h)
    text_pack_window_kb: int = 256     # that window, per source thread
    ingest_parse: bool = True          # GPU ingest: parse each fetch's records into an fp32 image
                                       # arena right behind its counting launch, so the batch
                                       # step of a whole-network plan (LeNet-5, ResNet-20) runs
                                       # the forward only (images through a pointer table)
    # parallelism (R3)
    workers: int = 8                   # NUM_WORKERS: placement only (one process per GPU here)
    source_parallelism: int = 2        # KAFKA_SPOUT_PARAL
    replicas: int = 0                  # INFERENCE_BOLT_PARAL; 0 = one per visible GPU
    sink_parallelism: int = 2          # KAFKA_BOLT_PARAL
    gpus: int = 0                      # GPUs to use (0 = all visible)
    numa_pin: bool = True              # a process serving ONE GPU pins its threads to that
                                       # GPU's NUMA node (gale.utils.pin_to_gpu_numa)
    locality_split: int = 1            # locality slots per GPU (single process): K slots on one
                                       # device, each with its own sources, batcher, pinned
                                       # pool + device mirror; a slot's idle replicas steal from
                                       # the others and parse stolen text from host-pinned
                                       # memory, as across GPUs (the multi-GPU dispatch on 1 GPU)
    # sink (R9, E7-E9)
    acks: int = 1                      # MainTopology.java:113
    sink_mode: str = "async"           # KafkaBolt async / sync / fire-and-forget
    # delivery of outputs: at-most-once = the reference (a failed send fails the unanchored tuple,
    # nothing replays it, KafkaBolt.java:133-137); at-least-once = an output that is never
    # acknowledged keeps its input offset uncommitted and the rank exits non-zero to be respawned
    # from the committed offsets; auto = at-least-once when offsets are resumed (start_offset
    # committed or group membership), else at-most-once
    delivery: str = "auto"
    producer_retries: int = 3          # kafka-clients retries (0.11 default 0): retriable produce
                                       # errors are re-sent after retry_backoff_ms
    retry_backoff_ms: int = 100        # retry.backoff.ms
    delivery_timeout_ms: int = 120000  # delivery.timeout.ms: no retry after this long
    value_format: str = "json"         # json-string = spring JsonSerializer double encoding
    type_id_header: bool = False       # add __TypeId__: java.lang.String (spring JsonSerializer)
    linger_ms: int = 0
    compression: str = "none"          # sink compression.type: none | gzip | snappy | lz4 | zstd
                                       # (kafka-clients default none; the input side decodes
                                       # every codec and the old message formats regardless)
    on_error: str = "null"             # reference: malformed input -> null record
    output_key: str = "none"           # reference: unkeyed output (E9); "input" = input's key
    float_format: str = "jdk19"        # prediction digits: jdk19 = shortest round-trip (GPU
                                       # formatted); java8 = the reference runtime's
                                       # Float.toString (host formatted, csrc/codec/java8_float.cpp)
    producer_buffer_mb: int = 32       # unsent output bytes per sink producer before the sink
                                       # blocks (Kafka buffer.memory, 32 MB default)
    producer_request_kb: int = 1024    # bytes per produce request (Kafka max.request.size)
    output_partition: int = -1         # -1: the producer's partitioner (reference: unkeyed
                                       # round-robin); >= 0: every output record to this
                                       # partition (e.g. the one this process's broker leads)
    # lifetime (reference: sleep 1 h then kill, MainTopology.java:71-77)
    duration: float = 3600.0
    # model / compute
    model: str = "resnet20"
    dtype: str = "bf16"
    weights: str = ""                  # .npz / .safetensors (torch layout); empty = seeded init
    seed: int = 0
    max_batch: int = 256
    max_wait_us: int = 2000
    slo_p99_ms: float = 0.0            # latency-SLO mode (config 5): adapt batch/wait to a p99
    queue_depth: int = 8192
    use_graph: bool = True
    graph_step: bool = True            # whole-network plans: each batch step (metadata H2D,
                                       # parse, forward, format, status D2H) is ONE replay of a
                                       # per-slot captured hipGraph (else launched op by op)
    gpu_wait_poll_us: int = 20         # > 0: replicas sleep-poll their batch events (0: spin)
    step_launch: str = "direct"        # the kernels-only batch step (parse -> forward) launched
                                       # kernel by kernel ("direct") or as a hipGraph replay
                                       # ("graph": the runtime's graph-launch bookkeeping kept a
                                       # helper thread spinning at ~0.8 of a core,
                                       # profiles/r5_ab_step_launch.jsonl)
    replica_priority: str = "normal"   # high: replica streams at the top stream priority (their
                                       # step kernels dispatch ahead of the GPU ingest's)
    gpu_encode: bool = True            # prediction text (Float.toString) formatted on the GPU
    fold_bn: bool = True               # False: standalone BatchNorm kernels (bf16 / fp32)
    stub: bool = False                 # CPU stub replicas (plumbing without a GPU)
    stub_null: bool = False            # stub replicas skip parsing/compute (host-path benchmark)
    stub_delay_us: int = 0             # stub replicas: emulated device time per batch
    # robustness / observability
    watchdog_ms: int = 30000
    # supervisor (Storm supervisors restart dead workers): a replica that failed is
    # recovered and rejoins after restart_backoff_ms, up to max_restarts times (0 = stays dead)
    max_restarts: int = 3
    restart_backoff_ms: int = 500
    # rank supervisor (gale/supervisor.py; Storm supervisors respawn dead worker JVMs,
    # MainTopology.java:25,65-66): > 0 = this command starts and supervises that many rank
    # processes (one per GPU), respawning a dead one after rank_restart_backoff_ms, at most
    # rank_max_restarts times per rank (-1 = always)
    ranks: int = 0
    rank_max_restarts: int = 10
    rank_restart_backoff_ms: int = 1000
    rank_start_timeout_s: float = 300.0
    # more ranks than GPUs (a 1-GPU rehearsal of the multi-rank path): rank r serves GPU
    # r % device_count and the process group is gloo (RCCL refuses two ranks on one device)
    shared_gpu_rehearsal: bool = False
    fault: str = ""                    # replica_crash@N,parse_error@P,producer_fail@P
    trace: bool = False                # roctx ranges around pipeline stages (rocprofv3)
    profile: str = ""                  # run under rocprofv3 --kernel-trace --marker-trace --stats
    metrics_interval: float = 10.0
    metrics_file: str = ""             # JSON lines; empty = stderr
    metrics_port: int = -1             # >= 0: HTTP /metrics (Prometheus) + /stats (JSON) on
                                       # 127.0.0.1:port+local_rank (0 = any free port); -1 off
    log_level: str = "INFO"
    registry_dir: str = field(default_factory=lambda: os.path.join(
        os.path.expanduser("~"), ".gale", "topologies"))

    def validate(self) -> "GaleConfig":
        if self.producer_request_kb < 1:
            raise ValueError("--producer-request-kb must be >= 1")
        if self.producer_buffer_mb < 1:
            raise ValueError("--producer-buffer-mb must be >= 1")
        if self.output_partition < -1:
            raise ValueError("--output-partition must be -1 (partitioner) or a partition index")
        for k, allowed in CHOICES.items():
            v = getattr(self, k)
            if v not in allowed:
                raise ValueError(f"{k}={v!r}: expected one of {allowed}")
        if self.acks not in (0, 1, -1):
            raise ValueError("acks must be 0, 1 or -1")
        for k in ("source_parallelism", "sink_parallelism", "max_batch", "queue_depth"):
            if getattr(self, k) <= 0:
                raise ValueError(f"{k} must be positive")
        if self.group_membership and not (0 < self.heartbeat_interval_ms
                                          < self.session_timeout_ms):
            raise ValueError("group membership: need 0 < heartbeat_interval_ms < "
                             "session_timeout_ms")
        if self.slo_p99_ms < 0:
            raise ValueError("slo_p99_ms must be >= 0")
        if self.replicas < 0 or self.gpus < 0:
            raise ValueError("replicas/gpus must be >= 0")
        if self.ranks < 0 or self.rank_restart_backoff_ms < 0:
            raise ValueError("--ranks / --rank-restart-backoff-ms must be >= 0")
        if self.producer_retries < 0 or self.retry_backoff_ms < 0 or self.delivery_timeout_ms < 1:
            raise ValueError("--producer-retries / --retry-backoff-ms must be >= 0, "
                             "--delivery-timeout-ms >= 1")
        if self.effective_delivery == "at-least-once" and self.sink_mode == "fire-and-forget":
            raise ValueError("at-least-once delivery needs acknowledged sends: --sink-mode "
                             "async|sync (or --delivery at-most-once)")
        if self.locality_split < 1:
            raise ValueError("locality_split must be >= 1")
        if not self.topology_name:
            raise ValueError("topology name is required")
        if not self.fold_bn and self.dtype == "fp8":
            raise ValueError("--no-fold-bn (standalone BatchNorm plan) is bf16 / fp32 only")
        return self

    @property
    def effective_group(self) -> str:
        return self.group_id or self.topology_name

    @property
    def effective_delivery(self) -> str:
        if self.delivery != "auto":
            return self.delivery
        resumes = self.start_offset == "committed" or self.group_membership
        return "at-least-once" if resumes and self.sink_mode != "fire-and-forget" \
            else "at-most-once"

    def engine_dict(self, H: int, W: int, C: int, classes: int) -> Dict[str, Any]:
        """Keyword dict for the native ``gale._C.Engine``."""
        return dict(
            bootstrap=self.bootstrap, input_topic=self.input_topic, output_topic=self.output_topic,
            group_id=self.effective_group, client_id=self.topology_name,
            partitions=[int(p) for p in self.partitions.split(",") if p.strip()],
            source_parallelism=self.source_parallelism, start_offset=self.start_offset,
            auto_offset_reset=self.auto_offset_reset, delivery=self.effective_delivery,
            producer_retries=self.producer_retries, retry_backoff_ms=self.retry_backoff_ms,
            delivery_timeout_ms=self.delivery_timeout_ms,
            commit_interval_ms=self.commit_interval_ms, sink_parallelism=self.sink_parallelism,
            fetch_min_bytes=self.fetch_min_bytes, fetch_max_wait_ms=self.fetch_max_wait_ms,
            recv_lowat=self.recv_lowat_kb << 10 if self.recv_lowat_kb >= 0 else -1,
            fetch_max_bytes=self.fetch_max_kb << 10,
            partition_max_bytes=self.partition_max_kb << 10,
            pinned_fetch_bytes=self.pinned_fetch_mb << 20,
            group_membership=self.group_membership, session_timeout_ms=self.session_timeout_ms,
            rebalance_timeout_ms=self.rebalance_timeout_ms,
            heartbeat_interval_ms=self.heartbeat_interval_ms, assignor=self.assignor,
            lag_rebalance_records=self.lag_rebalance_records,
            rebalance_cooldown_ms=self.rebalance_cooldown_ms,
            decode_threads=self.decode_threads, check_crcs=self.check_crcs,
            text_pack=bool(self.gpu_ingest and self.text_pack and _pack_fast()),
            text_pack_bounce=self.text_pack_bounce, text_pack_window_kb=self.text_pack_window_kb,
            acks=self.acks, sink_mode=self.sink_mode, linger_ms=self.linger_ms,
            compression=self.compression,
            value_format=self.value_format, type_id_header=self.type_id_header,
            on_error=self.on_error, output_key=self.output_key, float_format=self.float_format,
            output_partition=self.output_partition,
            producer_buffer_bytes=self.producer_buffer_mb << 20,
            producer_request_bytes=self.producer_request_kb << 10, H=H, W=W, C=C, classes=classes,
            max_batch=self.max_batch,
            max_wait_us=self.max_wait_us, slo_p99_ms=self.slo_p99_ms,
            queue_depth=self.queue_depth,
            watchdog_ms=self.watchdog_ms, max_restarts=self.max_restarts,
            restart_backoff_ms=self.restart_backoff_ms, fault=self.fault, seed=self.seed,
            trace=self.trace)


def _pack_fast() -> bool:
    from gale._native import native

    return bool(native().text_pack_fast())


def _coerce(f: dataclasses.Field, raw: Any) -> Any:
    t = f.type if isinstance(f.type, str) else getattr(f.type, "__name__", str(f.type))
    if t == "bool":
        if isinstance(raw, bool):
            return raw
        s = str(raw).strip().lower()
        if s in ("1", "true", "yes", "on"):
            return True
        if s in ("0", "false", "no", "off", ""):
            return False
        raise ValueError(f"{f.name}: not a boolean: {raw!r}")
    if t == "int":
        return int(raw)
    if t == "float":
        return float(raw)
    return str(raw)


def from_sources(cli: Optional[Dict[str, Any]] = None, env: Optional[Dict[str, str]] = None,
                 toml_path: Optional[str] = None) -> GaleConfig:
    """Merge defaults < TOML < env (GALE_*) < CLI (only keys explicitly given)."""
    env = os.environ if env is None else env
    values: Dict[str, Any] = {}
    known = {f.name: f for f in fields(GaleConfig)}
    if toml_path:
        import tomli

        with open(toml_path, "rb") as fh:
            data = tomli.load(fh)
        data = data.get("gale", data)
        for k, v in data.items():
            k = k.replace("-", "_")
            if k not in known:
                raise ValueError(f"{toml_path}: unknown key {k!r}")
            values[k] = _coerce(known[k], v)
    for name, f in known.items():
        ev = env.get("GALE_" + name.upper())
        if ev is not None:
            values[name] = _coerce(f, ev)
    for k, v in (cli or {}).items():
        if v is None:
            continue
        if k not in known:
            raise ValueError(f"unknown option {k!r}")
        values[k] = _coerce(known[k], v)
    return GaleConfig(**values).validate()


def field_names() -> List[str]:
    return [f.name for f in fields(GaleConfig)]
