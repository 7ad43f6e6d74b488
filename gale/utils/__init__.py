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


def core_groups(cpus, sysfs: str = "/sys/devices/system/cpu") -> list:
    """The CPUs of ``cpus`` grouped by physical core (SMT siblings together), cores ordered by
    their lowest CPU id: [[0, 128], [1, 129], ...] on a 2-way SMT EPYC. A CPU whose topology
    cannot be read is its own core."""
    cpus = set(cpus)
    seen, out = set(), []
    for c in sorted(cpus):
        if c in seen:
            continue
        try:
            with open(f"{sysfs}/cpu{c}/topology/thread_siblings_list") as f:
                sib = sorted(_parse_cpulist(f.read()) & cpus)
        except (OSError, ValueError):
            sib = [c]
        if c not in sib:
            sib = [c] + sib
        seen.update(sib)
        out.append(sib)
    return out


def numa_slice(cpus, slot: int, cpus_per_rank: int, smt: bool = False,
               sysfs: str = "/sys/devices/system/cpu") -> set:
    """Slot ``slot``'s disjoint share of a NUMA node's CPUs.

    * ``smt=False``: the ``cpus_per_rank`` lowest CPU ids after the earlier slots' (physical
      cores before their SMT siblings on Linux's numbering);
    * ``smt=True``: whole physical cores with their SMT siblings, ``cpus_per_rank`` hardware
      threads per slot (16 cores + 16 siblings for 32): what each of 4 ranks on a 64-core,
      128-thread socket owns, and the slice a loopback sender and receiver can share a core's
      L2 in.

    Returns an empty set when the node has fewer CPUs than the slot needs."""
    if cpus_per_rank <= 0:
        return set(cpus)
    if not smt:
        ordered = sorted(cpus)
        part = ordered[slot * cpus_per_rank:(slot + 1) * cpus_per_rank]
        return set(part) if len(part) == cpus_per_rank else set()
    cores = core_groups(cpus, sysfs)
    tpc = max(1, max(len(g) for g in cores)) if cores else 1
    ncores = max(1, cpus_per_rank // tpc)
    part = cores[slot * ncores:(slot + 1) * ncores]
    if len(part) < ncores:
        return set()
    return {c for g in part for c in g}


def plan_rank_slices(gpu_nodes, node_cpus: dict, smt: bool = True,
                     sysfs: str = "/sys/devices/system/cpu") -> list:
    """Disjoint host CPU slices for the ranks of one node: ``gpu_nodes[i]`` is the NUMA node of
    rank i's GPU, ``node_cpus`` maps a node to its CPUs. The ranks on a node split it evenly,
    in rank order, as whole physical cores with their SMT siblings (``smt``) - on a 2-socket
    64-core EPYC with 4 GPUs per socket, 16 cores + 16 siblings per rank, each slice inside
    its own L3 domains. A rank whose node is unknown (-1) gets an empty set (left unpinned)."""
    out = []
    for i, node in enumerate(gpu_nodes):
        cpus = node_cpus.get(node, set())
        peers = [j for j, n in enumerate(gpu_nodes) if n == node]
        if node < 0 or not cpus:
            out.append(set())
            continue
        per = len(cpus) // len(peers)
        if smt:
            cores = core_groups(cpus, sysfs)
            tpc = max(len(g) for g in cores)
            per = (per // tpc) * tpc
        out.append(numa_slice(cpus, peers.index(i), per, smt, sysfs) if per > 0 else set())
    return out


def node_cpus(node: int) -> set:
    """CPUs of a NUMA node within this process's affinity (empty when unknown)."""
    if node < 0:
        return set()
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            return _parse_cpulist(f.read()) & os.sched_getaffinity(0)
    except OSError:
        return set()


def pin_cpus(cpus) -> set:
    """Restrict this process's future threads to ``cpus`` (no-op when empty)."""
    cpus = set(cpus)
    if cpus:
        os.sched_setaffinity(0, cpus)
    return cpus


def pin_to_gpu_numa(device: int, cpus_per_rank: int = 0, smt: bool = False) -> set:
    """Restrict this process's future threads to the CPUs of the GPU's NUMA node (within the
    current affinity). The host pipeline moves ~35 KB of JSON per image through fetch buffers
    that are DMA sources for this GPU: keeping its threads and their first-touch memory on the
    GPU's socket avoids cross-socket copies. ``cpus_per_rank`` > 0 narrows it to this GPU's
    own slice of the node (``numa_slice``: lowest CPU ids, or whole cores with their SMT
    siblings with ``smt``; GPUs of one node take disjoint slices in device order), so the
    threads stop migrating over the whole socket. Returns the CPU set used (empty: left
    unpinned). Call before the engine starts its threads (they inherit the creator's
    affinity)."""
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
        part = numa_slice(cpus, slot, cpus_per_rank, smt)
        if part:
            cpus = part
    if cpus:
        os.sched_setaffinity(0, cpus)
    return cpus


def thread_ctx_switches() -> dict:
    """Voluntary / involuntary context switches of this process's live threads, summed per
    pipeline stage: {stage: [voluntary, involuntary]} (``/proc/self/task/<tid>/status``). A
    voluntary switch is a thread blocking (a wake-up per socket read, queue wait or poll
    sleep); an involuntary one is preemption by another runnable thread - the cost of more
    runnable threads than CPUs in the slice."""
    out = {g: [0, 0] for _, g in THREAD_GROUPS}
    out["other"] = [0, 0]
    base = "/proc/self/task"
    for tid in os.listdir(base):
        try:
            with open(f"{base}/{tid}/status") as f:
                txt = f.read()
        except OSError:
            continue
        name, vol, inv = "", 0, 0
        for ln in txt.splitlines():
            if ln.startswith("Name:"):
                name = ln.split(None, 1)[1] if len(ln.split(None, 1)) > 1 else ""
            elif ln.startswith("voluntary_ctxt_switches:"):
                vol = int(ln.split()[1])
            elif ln.startswith("nonvoluntary_ctxt_switches:"):
                inv = int(ln.split()[1])
        group = next((g for pre, g in THREAD_GROUPS if name.startswith(pre)), "other")
        out[group][0] += vol
        out[group][1] += inv
    return out


def cpu_time_split(cpus) -> dict:
    """Seconds per /proc/stat category summed over ``cpus`` (all CPUs when empty): user, system,
    irq, softirq, idle. Loopback TCP receive processing runs as softirq on the sending CPU (or
    in ksoftirqd when deferred), outside any thread's utime/stime of this process."""
    tick = os.sysconf("SC_CLK_TCK")
    want = set(cpus) if cpus else None
    keys = ("user", "nice", "system", "idle", "iowait", "irq", "softirq")
    out = {k: 0.0 for k in keys}
    try:
        with open("/proc/stat") as f:
            for ln in f:
                if not ln.startswith("cpu") or ln.startswith("cpu "):
                    continue
                parts = ln.split()
                c = int(parts[0][3:])
                if want is not None and c not in want:
                    continue
                for k, v in zip(keys, parts[1:8]):
                    out[k] += int(v) / tick
    except (OSError, ValueError):
        return {}
    return out


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
