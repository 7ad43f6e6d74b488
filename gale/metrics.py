"""Metrics: a periodic JSON-lines reporter and a live HTTP endpoint.

Replaces what the reference gets from Storm UI (per-component latency / capacity /
emitted / acked / failed, E4) and the KafkaSpout ``kafkaOffset`` metric (E1).

* ``Reporter``: every interval one line with the interval's throughput (images/s, records/s),
  cumulative counters, per-stage latency quantiles from the engine's native histograms, queue
  depth and replica health, to stderr or a file.
* ``MetricsServer`` (``--metrics-port``): the same numbers on demand, like Storm UI's REST API -
  ``GET /metrics`` in the Prometheus text format (engine counters/gauges, per replica and per
  input partition series), ``GET /stats`` as one JSON document.
"""

from __future__ import annotations

import json
import math
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Dict, List, Optional, TextIO

KEYS = ("records_in", "records_out", "images_out", "errors", "produce_failures", "dropped",
        "requeued", "replica_failures", "replica_restarts", "queue_records", "replicas_alive",
        "commits", "lag_records", "lag_records_max", "fetch_lag_records",
        "e2e_us_p50", "e2e_us_p99", "queue_us_p50", "device_us_p50", "device_us_p99",
        "record_e2e_ms_p50", "record_e2e_ms_p99", "batch_images_mean", "rebalances",
        "generation", "assigned_partitions", "eff_max_batch", "eff_max_wait_us",
        "lag_rebalances", "lag_rebalances_skipped", "capacity_rps", "steals",
        "converted_batches", "poison_batches", "poison_records", "poison_unknown_span",
        "split_records",
        "graph_step_batches", "sparse_fetches", "restored_fetches", "pinned_chunks",
        "pinned_waits", "pinned_heap_budget")


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


def _label_str(labels: dict) -> str:
    if not labels:
        return ""
    esc = (lambda v: str(v).replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n"))
    return "{" + ",".join(f'{k}="{esc(v)}"' for k, v in sorted(labels.items())) + "}"


def prometheus_text(stats: dict, replicas: List[dict], partitions: List[dict],
                    labels: Optional[dict] = None) -> str:
    """Prometheus exposition (text format 0.0.4) of an engine snapshot: every numeric engine
    stat as ``gale_<name>``, replica health/work as ``gale_replica_<name>{replica=..}``, the
    kafkaOffset equivalent as ``gale_partition_<name>{partition=..}``."""
    base = dict(labels or {})
    fams: Dict[str, list] = {}  # metric family -> samples (grouped, as the format requires)

    def emit(name: str, value, extra: Optional[dict] = None):
        if isinstance(value, bool):
            value = int(value)
        if not isinstance(value, (int, float)) or (isinstance(value, float)
                                                    and not math.isfinite(value)):
            return
        fams.setdefault(name, []).append(f"{name}{_label_str(dict(base, **(extra or {})))} "
                                         f"{value}")

    for k in sorted(stats):
        emit(f"gale_{k}", stats[k])
    for i, r in enumerate(replicas):
        for k in sorted(r):
            if k != "name":
                emit(f"gale_replica_{k}", r[k], {"replica": i, "name": r.get("name", "")})
    for o in partitions:
        for k in sorted(o):
            if k != "partition":
                emit(f"gale_partition_{k}", o[k], {"partition": o["partition"]})
    lines = []
    for name, samples in fams.items():
        lines.append(f"# TYPE {name} gauge")
        lines.extend(samples)
    return "\n".join(lines) + "\n"


class MetricsServer:
    """Live metrics over HTTP on ``host:port`` (port 0 picks a free one: see ``.port``)."""

    def __init__(self, engine, port: int = 0, host: str = "127.0.0.1",
                 labels: Optional[dict] = None):
        self.engine = engine
        self.labels = dict(labels or {})
        srv = self

        class Handler(BaseHTTPRequestHandler):
            def log_message(self, *args):  # quiet
                pass

            def do_GET(self):
                try:
                    if self.path.startswith("/metrics"):
                        body = prometheus_text(srv.engine.stats(), srv.engine.replica_stats(),
                                               srv.engine.partition_offsets(), srv.labels)
                        ctype = "text/plain; version=0.0.4"
                    elif self.path.startswith("/stats"):
                        body = json.dumps({**srv.labels, "stats": srv.engine.stats(),
                                           "replicas": srv.engine.replica_stats(),
                                           "partitions": srv.engine.partition_offsets()})
                        ctype = "application/json"
                    else:
                        self.send_error(404)
                        return
                except Exception as e:  # never take the topology down
                    self.send_error(500, str(e))
                    return
                data = body.encode()
                self.send_response(200)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

        self._httpd = ThreadingHTTPServer((host, port), Handler)
        self._httpd.daemon_threads = True
        self.port = self._httpd.server_address[1]
        self._thread = threading.Thread(target=self._httpd.serve_forever, name="gale-http",
                                        daemon=True)

    def start(self) -> "MetricsServer":
        self._thread.start()
        return self

    def stop(self) -> None:
        self._httpd.shutdown()
        self._httpd.server_close()


def _match_appends(append_log, ack_log):
    """For each acknowledged record, the append time of the producer batch that holds its
    offset: returns (ack indices, append t_ns) for the matched records."""
    import numpy as np

    ap, abase, an, at = (np.asarray(x) for x in append_log)
    kp, koff = np.asarray(ack_log[0]), np.asarray(ack_log[1])
    idx, tapp = [], []
    for p in np.unique(kp):
        sel = ap == p
        if not sel.any():
            continue
        base, n, t = abase[sel], an[sel], at[sel]
        order = np.argsort(base)
        base, n, t = base[order], n[order], t[order]
        ks = np.nonzero(kp == p)[0]
        off = koff[ks]
        i = np.searchsorted(base, off, side="right") - 1
        ok = (i >= 0)
        i = np.clip(i, 0, len(base) - 1)
        ok &= off < base[i] + n[i]
        idx.append(ks[ok])
        tapp.append(t[i[ok]])
    if not idx:
        return np.zeros(0, dtype=np.int64), np.zeros(0, dtype=np.int64)
    return np.concatenate(idx), np.concatenate(tapp)


def append_to_ack_us(append_log, ack_log, with_ack_time=False):
    """Record-level latency (microseconds) from a producer's append log and the engine's ack
    log, both on CLOCK_MONOTONIC: ``append_log`` = (partition, base_offset, records, t_ns) per
    appended batch (``kafka.RateFeeder.take_log``), ``ack_log`` = (partition, offset, t_ns, ...)
    per acknowledged output (``Engine.take_ack_log``). Each acknowledged record is matched to
    the batch that contains its offset; records appended outside the log are skipped. With
    ``with_ack_time`` returns (latencies, ack t_ns) so a tail can be placed in time."""
    import numpy as np

    idx, tapp = _match_appends(append_log, ack_log)
    tack = np.asarray(ack_log[2])[idx]
    lat = (tack - tapp) / 1e3
    return (lat, tack) if with_ack_time else lat


def latency_stages_us(append_log, ack_log):
    """Per-record split of append -> ack into the pipeline stages (microseconds), from an ack
    log with stage times (``Engine.take_ack_log``: t_ack, t_fetch, t_take, t_done):
    broker_source = append -> fetch response received (broker residency, fetch wait, socket),
    queue = fetch -> batch dispatched (decode / GPU ingest and batching), replica = dispatch ->
    device done (H2D, parse, forward, D2H, completion wait), sink = done -> produce ack
    (prediction text, produce request, broker ack). With a t_ready column (ack logs of round 6 on)
    queue is also split into ingest = fetch -> handed to the batcher (CRC / count [/ parse] on
    the GPU, or the host decode) and batching = handed -> dispatched; queue = ingest + batching.
    Records without stage times are skipped."""
    import numpy as np

    idx, tapp = _match_appends(append_log, ack_log)
    tack, tf, tt, td = (np.asarray(ack_log[k])[idx] for k in (2, 3, 4, 5))
    tr = np.asarray(ack_log[6])[idx] if len(ack_log) > 6 else None
    ok = (tf > 0) & (tt > 0) & (td > 0)
    if tr is not None:
        ok &= tr > 0
        tr = tr[ok]
    tapp, tack, tf, tt, td = tapp[ok], tack[ok], tf[ok], tt[ok], td[ok]
    out = {"broker_source": (tf - tapp) / 1e3, "queue": (tt - tf) / 1e3,
           "replica": (td - tt) / 1e3, "sink": (tack - td) / 1e3}
    if tr is not None:
        out["ingest"] = (tr - tf) / 1e3
        out["batching"] = (tt - tr) / 1e3
    return out
