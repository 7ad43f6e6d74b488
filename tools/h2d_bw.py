"""Host->device copy bandwidth from pinned memory (the GPU-ingest path's link), 1 and 4 streams."""
import json

import torch

n = 64 << 20
h = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device="cuda")
res = {}
for streams in (1, 4):
    ss = [torch.cuda.Stream() for _ in range(streams)]
    chunk = n // streams
    for _ in range(3):
        for i, s in enumerate(ss):
            with torch.cuda.stream(s):
                d[i * chunk:(i + 1) * chunk].copy_(h[i * chunk:(i + 1) * chunk], non_blocking=True)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 20
    a.record()
    for _ in range(it):
        for i, s in enumerate(ss):
            s.wait_event(a) if False else None
            with torch.cuda.stream(s):
                d[i * chunk:(i + 1) * chunk].copy_(h[i * chunk:(i + 1) * chunk], non_blocking=True)
    for s in ss:
        torch.cuda.current_stream().wait_stream(s)
    b.record()
    torch.cuda.synchronize()
    res[f"h2d_GBps_{streams}stream"] = round(n * it / (a.elapsed_time(b) / 1e3) / 1e9, 1)
print(json.dumps(res))
