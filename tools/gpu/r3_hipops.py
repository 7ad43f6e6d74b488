"""Per HIP operation, the CPU the runtime's own threads spend (the unnamed busy thread of a
serving process): each op is issued 20k times from this thread, then the per-thread CPU of the
other threads over that window is listed."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def threads():
    out = {}
    for t in os.listdir("/proc/self/task"):
        try:
            st = open(f"/proc/self/task/{t}/stat").read()
        except OSError:
            continue
        rp = st.rindex(")")
        f = st[rp + 2:].split()
        out[int(t)] = (st[st.index("(") + 1:rp], int(f[11]) + int(f[12]))
    return out


me = ctypes.CDLL(None).syscall(186)  # gettid


def measure(tag, fn, n=20000):
    a = threads()
    t0 = time.perf_counter()
    fn(n)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    b = threads()
    hot = {t: (b[t][0], round((b[t][1] - a[t][1]) / 100 / dt, 2)) for t in b
           if t in a and t != me and b[t][1] - a[t][1] > 2}
    print(f"{tag}: {n / dt:.0f} ops/s, other threads' cores: {hot}", flush=True)


torch.cuda.init()
s = torch.cuda.Stream()
stream = ctypes.c_void_p(s.cuda_stream)
h = torch.empty(1 << 20, dtype=torch.uint8).pin_memory()
d = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
ev = ctypes.c_void_p()
hip.hipEventCreateWithFlags(ctypes.byref(ev), 2)  # hipEventDisableTiming


def h2d(n):
    for _ in range(n):
        hip.hipMemcpyAsync(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(h.data_ptr()),
                           ctypes.c_size_t(65536), 1, stream)


def d2h(n):
    for _ in range(n):
        hip.hipMemcpyAsync(ctypes.c_void_p(h.data_ptr()), ctypes.c_void_p(d.data_ptr()),
                           ctypes.c_size_t(4096), 2, stream)


def record_query(n):
    for _ in range(n):
        hip.hipEventRecord(ev, stream)
        while hip.hipEventQuery(ev) != 0:
            pass


def kernel(n):
    with torch.cuda.stream(s):
        for _ in range(n):
            d.add_(1)


measure("idle", lambda n: time.sleep(1.0))
measure("H2D 64KB pinned", h2d)
measure("D2H 4KB pinned", d2h)
measure("event record+query", record_query)
measure("kernel launch", kernel)


g = torch.cuda.CUDAGraph()
x = torch.zeros(1 << 16, device="cuda")
with torch.cuda.graph(g):
    for _ in range(8):
        x.add_(1)


def graph(n):
    for _ in range(n):
        g.replay()


measure("graph replay (8 kernels)", graph)


def graph_query(n):
    for _ in range(n):
        g.replay()
        hip.hipEventRecord(ev, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        while hip.hipEventQuery(ev) != 0:
            pass


measure("graph replay + event record/query", graph_query)
