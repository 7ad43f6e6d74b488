"""Small host-side helpers shared by the CLI, the benchmark and the tools."""

from __future__ import annotations

import os
import socket


def cgroup_cpu_quota() -> float:
    """The cgroup v2 CPU bandwidth quota in CPUs (cpu.max), 0.0 when unlimited or unknown."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        return 0.0 if quota == "max" else int(quota) / int(period)
    except (OSError, ValueError):
        return 0.0


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


def _parse_cpulist(text: str) -> set:
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def gpu_numa_node(device: int) -> int:
    """NUMA node of a GPU (its PCI function's sysfs ``numa_node``), -1 when unknown."""
    from gale._native import native

    try:
        bdf = native().device_pci_bus_id(device).lower()
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            return int(f.read().strip())
    except (OSError, ValueError, RuntimeError):
        return -1


def pin_to_gpu_numa(device: int, cpus_per_rank: int = 0) -> set:
    """Restrict this process's future threads to the CPUs of the GPU's NUMA node (within the
    current affinity). The host pipeline moves ~35 KB of JSON per image through fetch buffers
    that are DMA sources for this GPU: keeping its threads and their first-touch memory on the
    GPU's socket avoids cross-socket copies. ``cpus_per_rank`` > 0 narrows it to this GPU's
    own slice of the node (lowest CPU ids first: physical cores before their SMT siblings;
    GPUs of one node take disjoint slices in device order), so the threads stop migrating over
    the whole socket. Returns the CPU set used (empty: left unpinned). Call before the engine
    starts its threads (they inherit the creator's affinity)."""
    node = gpu_numa_node(device)
    if node < 0:
        return set()
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            cpus = _parse_cpulist(f.read()) & os.sched_getaffinity(0)
    except OSError:
        return set()
    if cpus and cpus_per_rank > 0:
        slot = sum(1 for d in range(device) if gpu_numa_node(d) == node)
        ordered = sorted(cpus)
        part = ordered[slot * cpus_per_rank:(slot + 1) * cpus_per_rank]
        if len(part) == cpus_per_rank:
            cpus = set(part)
    if cpus:
        os.sched_setaffinity(0, cpus)
    return cpus


THREAD_GROUPS = (("gl-brk", "broker"), ("gl-src", "source"), ("gl-dec", "decode"),
                 ("gl-rep", "replica"), ("gl-sink", "sink"), ("gl-watchdog", "watchdog"))


def thread_cpu_by_thread() -> dict:
    """CPU seconds (user + system) per live thread of this process: {(tid, name): seconds}."""
    tick = os.sysconf("SC_CLK_TCK")
    out = {}
    base = "/proc/self/task"
    for tid in os.listdir(base):
        try:
            with open(f"{base}/{tid}/stat") as f:
                st = f.read()
        except OSError:
            continue
        lp, rp = st.index("("), st.rindex(")")
        rest = st[rp + 2:].split()
        out[(int(tid), st[lp + 1:rp])] = (int(rest[11]) + int(rest[12])) / tick
    return out


def thread_cpu_seconds() -> dict:
    """CPU seconds (user + system) of this process's live threads, summed per pipeline stage.

    The native threads name themselves (csrc/include/gale/thread_name.h: gl-src<i>, gl-dec<i>,
    gl-rep<i>, gl-sink, gl-brk-*); anything else (Python, HIP runtime, RCCL) is "other". Threads
    that exited between two snapshots drop out, so take deltas over a window in which the
    pipeline's threads stay alive."""
    tick = os.sysconf("SC_CLK_TCK")
    out = {g: 0.0 for _, g in THREAD_GROUPS}
    out["other"] = 0.0
    base = "/proc/self/task"
    for tid in os.listdir(base):
        try:
            with open(f"{base}/{tid}/stat") as f:
                st = f.read()
        except OSError:
            continue
        lp, rp = st.index("("), st.rindex(")")
        name = st[lp + 1:rp]
        rest = st[rp + 2:].split()
        sec = (int(rest[11]) + int(rest[12])) / tick  # fields 14, 15: utime, stime
        group = next((g for pre, g in THREAD_GROUPS if name.startswith(pre)), "other")
        out[group] += sec
    return out


def name_this_thread(name: str) -> None:
    """Set the calling thread's OS name (prctl PR_SET_NAME, <= 15 bytes) so per-thread CPU
    accounting (thread_cpu_seconds, bench.py --timeline) can tell Python threads apart."""
    import ctypes

    try:
        ctypes.CDLL(None).prctl(15, name.encode()[:15], 0, 0, 0)
    except (OSError, AttributeError):
        pass


def free_port(host: str = "127.0.0.1") -> int:
    """An ephemeral TCP port that was free a moment ago (embedded brokers, rendezvous)."""
    s = socket.socket()
    try:
        s.bind((host, 0))
        return s.getsockname()[1]
    finally:
        s.close()
