"""Periodic JSON-lines metrics reporter.

Replaces what the reference gets from Storm UI (per-component latency / capacity /
emitted / acked / failed, E4) and the KafkaSpout ``kafkaOffset`` metric (E1). Every interval it
writes one line with the interval's throughput (images/s, records/s), cumulative counters,
per-stage latency quantiles from the engine's native histograms, queue depth and replica
health, to stderr or a file.
"""

from __future__ import annotations

import json
import sys
import threading
import time
from typing import Callable, Dict, Optional, TextIO

KEYS = ("records_in", "records_out", "images_out", "errors", "produce_failures", "dropped",
        "requeued", "replica_failures", "replica_restarts", "queue_records", "replicas_alive",
        "commits", "lag_records", "lag_records_max", "fetch_lag_records",
        "e2e_us_p50", "e2e_us_p99", "queue_us_p50", "device_us_p50", "device_us_p99",
        "record_e2e_ms_p50", "record_e2e_ms_p99", "batch_images_mean", "rebalances",
        "generation", "assigned_partitions", "eff_max_batch", "eff_max_wait_us")


class Reporter:
    def __init__(self, stats_fn: Callable[[], Dict[str, float]], interval: float = 10.0,
                 out: Optional[TextIO] = None, path: str = "", labels: Optional[dict] = None,
                 extra_fn: Optional[Callable[[], dict]] = None):
        self.stats_fn = stats_fn
        self.extra_fn = extra_fn  # merged into every line (e.g. the owned input partitions)
        self.interval = interval
        self.labels = dict(labels or {})
        self._own = open(path, "a", buffering=1) if path else None
        self.out = self._own or out or sys.stderr
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._last: Optional[Dict[str, float]] = None
        self._last_t = 0.0

    def snapshot(self) -> dict:
        now = time.time()
        s = self.stats_fn()
        line = {"ts": round(now, 3), **self.labels}
        if self._last is not None and now > self._last_t:
            dt = now - self._last_t
            line["images_per_s"] = round((s["images_out"] - self._last["images_out"]) / dt, 1)
            line["records_per_s"] = round((s["records_out"] - self._last["records_out"]) / dt, 1)
        for k in KEYS:
            if k in s:
                v = s[k]
                line[k] = int(v) if float(v).is_integer() else round(v, 3)
        if self.extra_fn is not None:
            line.update(self.extra_fn())
        self._last, self._last_t = s, now
        return line

    def report(self) -> dict:
        line = self.snapshot()
        self.out.write(json.dumps(line) + "\n")
        self.out.flush()
        return line

    def _run(self):
        self.snapshot()
        while not self._stop.wait(self.interval):
            try:
                self.report()
            except Exception as e:  # the reporter must never take the topology down
                print(f"[gale metrics] {e}", file=sys.stderr)

    def start(self) -> "Reporter":
        if self.interval > 0:
            self._thread = threading.Thread(target=self._run, name="gale-metrics", daemon=True)
            self._thread.start()
        return self

    def stop(self, final: bool = True, close: bool = True) -> None:
        self._stop.set()
        if self._thread:
            self._thread.join()
        if final:
            try:
                self.report()
            except Exception:
                pass
        if close:
            self.close()

    def close(self) -> None:
        if self._own and not self._own.closed:
            self._own.close()
