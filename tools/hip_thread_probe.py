#!/usr/bin/env python3
"""Which HIP operation keeps the HIP/HSA runtime's helper thread busy?

The serving engine's busiest unnamed thread (bench.py --timeline "other_probe") spins in user
space at ~0.8 of a core. This drives one kind of operation at a fixed rate for 2 s per case and
reports the CPU seconds per second of every thread that is not the driving one:

  copy   small pinned H2D hipMemcpyAsync (SDMA) + event record / query, like the GPU ingest's
  kernel a small kernel launch + event record / query, like the replica step
  graph  a one-kernel hipGraph replay + event record / query
  idle   nothing (the baseline)
"""

import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gale.utils import thread_cpu_by_thread  # noqa: E402


def drive(kind, rate, seconds=2.0):
    s = torch.cuda.Stream()
    h = torch.empty(16384, dtype=torch.uint8).pin_memory()
    d = torch.empty(16384, dtype=torch.uint8, device="cuda")
    x = torch.ones(1024, device="cuda")
    g = None
    if kind == "graph":
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            x.mul_(1.0)
    me = threading.get_native_id()
    before = thread_cpu_by_thread()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds:
        due = t0 + n / rate
        while time.perf_counter() < due:
            pass
        with torch.cuda.stream(s):
            if kind == "copy":
                d.copy_(h, non_blocking=True)
            elif kind == "kernel":
                x.mul_(1.0)
            elif kind == "graph":
                g.replay()
            ev = torch.cuda.Event()
            if kind != "idle":
                ev.record(s)
        if kind != "idle":
            while not ev.query():
                time.sleep(20e-6)
        n += 1
    dt = time.perf_counter() - t0
    after = thread_cpu_by_thread()
    other = {f"{k[1]}:{k[0]}": round((v - before.get(k, 0.0)) / dt, 3)
             for k, v in after.items() if k[0] != me and v - before.get(k, 0.0) > 0.01}
    return {"case": kind, "rate_per_s": round(n / dt), "other_cores": other}


def main():
    torch.cuda.init()
    torch.ones(1, device="cuda")
    for kind in ("idle", "copy", "kernel", "graph"):
        for rate in (5000, 20000):
            print(json.dumps(drive(kind, rate)), flush=True)


if __name__ == "__main__":
    main()
