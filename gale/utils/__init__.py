"""Small host-side helpers shared by the CLI, the benchmark and the tools."""

from __future__ import annotations

import os
import socket


def host_cpus_per_rank() -> float:
    """CPUs this rank may use: min(affinity, cgroup CPU quota) / ranks on this node.

    The benchmark sizes its host pipeline (replicas per GPU, each with its own consumer, decode
    and sink share) from this: on a GPU box the whole machine's CPUs are visible through
    ``os.cpu_count()`` but the job only gets a cgroup share of them.
    """
    n = float(len(os.sched_getaffinity(0)))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, int(quota) / int(period))
    except (OSError, ValueError):
        pass
    return n / max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))


def free_port(host: str = "127.0.0.1") -> int:
    """An ephemeral TCP port that was free a moment ago (embedded brokers, rendezvous)."""
    s = socket.socket()
    try:
        s.bind((host, 0))
        return s.getsockname()[1]
    finally:
        s.close()
