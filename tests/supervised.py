"""Helpers for the supervised multi-rank tests (test_supervisor_cpu.py, test_supervisor_gpu.py).

A supervised job is ``python -m gale NAME IN OUT --ranks N ...`` started as a subprocess. Its
stderr (the supervisor's events plus every rank's log lines) goes to a FILE, never a pipe: a
pipe nobody drains until the end fills at 64 KiB and then blocks every rank that logs, which
stalls heartbeats and fetches mid-test. Ranks run with GALE_LOG_COMMITS=1, so on a failure the
test can print each rank's group generations and every offset commit next to the missing keys.
"""

from __future__ import annotations

import json
import os
import subprocess
import sys
import time
from typing import Dict, Iterable, List, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def wait_for(pred, timeout=30.0, step=0.05):
    t = time.time() + timeout
    while time.time() < t:
        if pred():
            return True
        time.sleep(step)
    return False


def lines(path) -> List[dict]:
    if not os.path.exists(path):
        return []
    out = []
    with open(path) as fh:
        for x in fh:
            x = x.strip()
            if x:
                try:
                    out.append(json.loads(x))
                except json.JSONDecodeError:  # (a line being written)
                    pass
    return out


def start_job(args: List[str], log_path) -> subprocess.Popen:
    env = dict(os.environ, OMP_NUM_THREADS="1", GALE_LOG_COMMITS="1")
    fh = open(log_path, "w")
    try:
        return subprocess.Popen([sys.executable, "-m", "gale", *args], cwd=ROOT,
                                stdout=subprocess.DEVNULL, stderr=fh, text=True, env=env)
    finally:
        fh.close()  # (the child holds its own descriptor)


def last_rows(metrics, incarnations: Dict[int, int] = None) -> Dict[int, dict]:
    """The latest metrics row of each rank (of the given incarnation per rank, if any)."""
    last: Dict[int, dict] = {}
    for r in lines(metrics):
        rk = r.get("rank")
        if rk is None:
            continue
        if incarnations and r.get("rank_restarts", 0) != incarnations.get(rk, 0):
            continue
        last[rk] = r
    return last


def ranks_serving(metrics, ranks: int, partitions: int, group: bool = True) -> bool:
    """Every rank reports partitions assigned (its sources have sought them), together covering
    all `partitions`, and - under group membership - all in the same generation. Appending
    input before this point races the ranks' first seek."""
    last = last_rows(metrics)
    if len(last) != ranks or any(r.get("assigned_partitions", 0) <= 0 for r in last.values()):
        return False
    parts = set()
    for r in last.values():
        parts |= set(r.get("partitions", []))
    if parts != set(range(partitions)):
        return False
    return not group or len({r.get("generation") for r in last.values()}) == 1


def read_keys(broker, topic: str, partitions: Iterable[int] = (0,)) -> Dict[bytes, bytes]:
    out = {}
    for p in partitions:
        for r in broker.read(topic, p):
            out[r["key"]] = r["value"]
    return out


def diagnose(broker, where: Dict[bytes, Tuple[int, int]], got: Iterable[bytes], group: str,
             topic: str, partitions: int, log_path, metrics=None) -> str:
    """Why keys are missing: each missing key's input (partition, offset), the group's committed
    offsets and log ends, each rank's `[gale group]` / `[gale commit]` / sink lines, and the
    last metrics row per rank."""
    missing = sorted(set(where) - set(got), key=lambda k: where[k])
    parts = []
    parts.append(f"{len(missing)} of {len(where)} keys missing")
    by_p: Dict[int, List[int]] = {}
    for k in missing:
        by_p.setdefault(where[k][0], []).append(where[k][1])
    for p in sorted(by_p):
        offs = by_p[p]
        parts.append(f"  partition {p}: {len(offs)} missing, offsets {offs[:12]}"
                     f"{' ...' if len(offs) > 12 else ''}")
    for p in range(partitions):
        try:
            parts.append(f"  partition {p}: committed {broker.committed(group, topic, p)} "
                         f"log_end {broker.log_end(topic, p)}")
        except Exception as e:  # noqa: BLE001 - diagnostics only
            parts.append(f"  partition {p}: {e}")
    try:
        with open(log_path, errors="replace") as fh:
            log = [x.rstrip() for x in fh if any(t in x for t in (
                "[gale group]", "[gale commit]", "[gale sink]", "[gale source", '"event"',
                "Error", "error"))]
    except OSError:
        log = []
    parts.append("rank log (group / commit / sink / events), last 120 lines:")
    parts += ["  " + x for x in log[-120:]]
    if metrics is not None:
        for rk, r in sorted(last_rows(metrics).items()):
            parts.append(f"  rank {rk} last metrics: " + json.dumps(
                {k: r.get(k) for k in ("rank_restarts", "generation", "assigned_partitions",
                                       "partitions", "records_in", "records_out", "commits",
                                       "produce_failures", "undelivered")}))
    return "\n".join(parts)
