"""Python face of the native serving engine (csrc/runtime/engine.cpp).

Builds the replicas a topology asks for and hands them to ``gale._C.Engine``:

* GPU replicas — one ``ModelReplica`` (packed weights + hipGraph plan executor) per replica,
  placed round-robin over the process's GPUs. Weights are materialised once per device: on the
  source rank from the seed (or a weights file) and RCCL-broadcast over xGMI to every other rank
  of the default process group (``gale.parallel.weights``); inside one process they are copied
  device-to-device. This replaces every InferenceBolt task loading its own SavedModel copy
  (InferenceBolt.java:48-58).
* stub replicas — the CPU plumbing replica (``--stub``), no GPU needed.

The hot path never returns to Python: source threads, micro-batcher, replica workers and sink
threads all run natively; Python only starts/stops the engine and reads its metrics.
"""

from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

from gale._native import native
from gale.config import GaleConfig
from gale.models import get_model


def device_cpus(device: int) -> set:
    """CPUs of the GPU's NUMA node within this process's affinity (empty when unknown)."""
    import os

    from gale.utils import _parse_cpulist, gpu_numa_node

    node = gpu_numa_node(device)
    if node < 0:
        return set()
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            return _parse_cpulist(f.read()) & os.sched_getaffinity(0)
    except OSError:
        return set()


def replica_devices(n_replicas: int, devices: Sequence[int]) -> List[int]:
    if not devices:
        raise ValueError("no devices to place replicas on")
    return [devices[i % len(devices)] for i in range(n_replicas)]


class Engine:
    def __init__(self, cfg: GaleConfig, devices: Optional[Sequence[int]] = None,
                 max_records: int = -1, params: Optional[dict] = None,
                 model_replicas: Optional[list] = None, stub_localities: Sequence[int] = ()):
        self.cfg = cfg
        self.net = get_model(cfg.model)
        H, W, C = self.net.input_shape
        d = cfg.engine_dict(H, W, C, self.net.classes)
        d["max_records"] = max_records
        self.model_replicas: list = []
        self.devices: List[int] = []
        if cfg.stub:
            self._native = native().Engine(d)
            for i in range(max(1, cfg.replicas)):
                loc = stub_localities[i % len(stub_localities)] if stub_localities else -1
                self._native.add_stub_replica(cfg.max_batch, cfg.stub_delay_us, not cfg.stub_null,
                                              loc)
            return
        if model_replicas is not None:
            reps = list(model_replicas)
        else:
            reps = self._build_gpu_replicas(devices, params)
        devs = sorted({r.device.index or 0 for r in reps}, key=[r.device.index or 0
                                                                for r in reps].index)
        # the GPU ingest parses each fetch into an image arena when every replica's batch step
        # can take the images from there: the direct-launch step of a whole-network plan with
        # the prediction text in its epilogue (GpuReplica ptr_input_)
        d["ingest_parse"] = bool(
            cfg.ingest_parse and cfg.gpu_ingest and cfg.use_graph and cfg.graph_step
            and cfg.gpu_encode and cfg.float_format == "jdk19" and cfg.step_launch == "direct"
            and reps and all(getattr(r.executor, "step_out_ok", False) for r in reps))
        if (len(devs) > 1 or cfg.locality_split > 1) and cfg.numa_pin:
            # single-process multi-GPU: each GPU's replica workers and sources run on the CPUs
            # of that GPU's NUMA node (its pinned fetch buffers are first-touched there)
            d["device_cpus"] = {dev: sorted(device_cpus(dev)) for dev in devs}
        self._native = native().Engine(d)
        per_dev: Dict[int, int] = {}
        k = max(1, cfg.locality_split)
        for rep in reps:
            dev = rep.device.index or 0
            j = per_dev.get(dev, 0)
            per_dev[dev] = j + 1
            # --locality-split K: the device's replicas are dealt over K locality slots
            loc = dev * k + (j % k) if k > 1 else -1
            # Java 8 digits are formatted on the host (the GPU formatter is the JDK 19 rule)
            self._native.add_gpu_replica(rep.executor, cfg.use_graph, cfg.gpu_wait_poll_us,
                                         cfg.gpu_encode and cfg.float_format == "jdk19", loc,
                                         cfg.graph_step, cfg.replica_priority == "high",
                                         cfg.step_launch == "direct")
            self.model_replicas.append(rep)
            self.devices.append(dev)
        if cfg.gpu_ingest:
            # fetch buffers of each device's sources are mirrored on that device once and
            # parsed in place
            # one lane (stream + staging) per thread that runs the ingest: the decode workers,
            # or the sources themselves when there are none
            lanes = cfg.decode_threads if cfg.decode_threads > 0 else cfg.source_parallelism
            # the lanes sleep-poll their fetch's completion every 20 us (GALE_INGEST_POLL_US, A/B)
            poll_us = int(os.environ.get("GALE_INGEST_POLL_US", "20"))
            for dev in devs:
                self._native.enable_gpu_ingest(dev, max(1, lanes), poll_us)

    def _build_gpu_replicas(self, devices: Optional[Sequence[int]], params: Optional[dict]):
        import torch

        from gale.parallel.weights import materialize_weights
        from gale.runtime.replica import ModelReplica

        if not torch.cuda.is_available():
            raise RuntimeError("no GPU visible: run with --stub for CPU plumbing replicas")
        if devices is None:
            n = torch.cuda.device_count()
            devices = list(range(n if self.cfg.gpus <= 0 else min(self.cfg.gpus, n)))
        n_rep = self.cfg.replicas if self.cfg.replicas > 0 else len(devices)
        wdtype = self.cfg.dtype  # bf16 | fp8 | fp32 (packed weight / activation type)
        if params is None and self.cfg.weights:
            from gale.models.weights_io import load_params

            params = load_params(self.cfg.weights, self.net)
        placement = replica_devices(n_rep, devices)
        used = sorted(set(placement), key=placement.index)
        src = materialize_weights(self.net, torch.device("cuda", used[0]), seed=self.cfg.seed,
                                  wdtype=wdtype, params=params, fold_bn=self.cfg.fold_bn)
        if len(used) > 1:  # one process, several GPUs: RCCL broadcast over xGMI
            from gale.parallel.weights import replicate_weights

            packed: Dict[int, "torch.Tensor"] = dict(zip(used, replicate_weights(src, used)))
        else:
            packed = {used[0]: src}
        reps = []
        for dev in placement:
            reps.append(ModelReplica(self.net, packed[dev], max_batch=self.cfg.max_batch,
                                     slots=3, wdtype=wdtype, fold_bn=self.cfg.fold_bn))
        for r in reps:
            r.capture()
        return reps

    # -- lifecycle ---------------------------------------------------------------------------
    def start(self) -> None:
        self._native.start()

    def stop(self) -> None:
        self._native.stop()

    def wait(self, timeout_s: Optional[float] = None) -> bool:
        return self._native.wait(-1 if timeout_s is None else int(timeout_s * 1000))

    def wait_completed(self, n: int, timeout_s: Optional[float] = None) -> bool:
        """Block until >= n records completed (the engine keeps running)."""
        return self._native.wait_completed(n, -1 if timeout_s is None else int(timeout_s * 1000))

    def last_wait(self):
        """(CLOCK_MONOTONIC ns, records completed) of the completion that reached the last
        wait_completed target, taken by the completing thread; (0, 0) if the target was already
        reached when the wait began."""
        return tuple(self._native.last_wait())

    @property
    def running(self) -> bool:
        return self._native.running

    @property
    def completed(self) -> int:
        return self._native.completed

    def stats(self) -> Dict[str, float]:
        return dict(self._native.stats())

    def replica_stats(self) -> List[dict]:
        return list(self._native.replica_stats())

    def partition_offsets(self) -> List[dict]:
        """storm-kafka ``kafkaOffset`` analogue: per input partition the log end (high
        watermark), next fetch offset, commit position and lag."""
        return list(self._native.partition_offsets())

    def reset_stats(self) -> None:
        self._native.reset_stats()

    def set_ack_log(self, on: bool, capacity: int = 8 << 20) -> None:
        """Log every acknowledged record (partition, offset, CLOCK_MONOTONIC ns) while on."""
        self._native.set_ack_log(on, capacity)

    def take_ack_log(self):
        """(partition, offset, t_ack_ns, t_fetch_ns, t_take_ns, t_done_ns, t_ready_ns) numpy
        arrays of the ack log (and clear it); all CLOCK_MONOTONIC. t_ready: decode / GPU ingest
        done, the record handed to the batcher."""
        return self._native.take_ack_log()
