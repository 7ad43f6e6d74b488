"""Host packing throughput of the nibble transport (csrc/codec/text_pack.h) by buffer size:
cache-resident vs DRAM-streaming passes over Jackson InstObj text."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gale._native import native  # noqa: E402

N = native()
x = np.random.default_rng(0).random((8, 32, 32, 3), dtype=np.float32)
doc = N.encode_instances(x)
for m in (1, 4, 16, 64, 256):
    d = doc * m
    dt, n = N.text_pack_bench(d, max(5, 400 // m), False)
    print(json.dumps({"kb": len(d) // 1024, "gb_s": round(len(d) / dt / 1e9, 2),
                      "ratio": round(n / len(d), 4), "vbmi": N.text_pack_fast()}))

if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "pinned":
    # same pass between pinned (hipHostMalloc via torch) and pageable buffers
    import torch

    d = doc * 64
    src_np = np.frombuffer(d, np.uint8)
    for kind in ("pageable", "pinned"):
        src = torch.from_numpy(src_np.copy())
        dst = torch.empty(len(d), dtype=torch.uint8)
        tab = torch.empty(len(d) // 256 + 16, dtype=torch.int32)
        if kind == "pinned":
            src, dst, tab = src.pin_memory(), dst.pin_memory(), tab.pin_memory()
        for sz in (256 << 10, 4 << 20, len(d)):
            dt, n = N.text_pack_bench_ptr(src.data_ptr(), sz, dst.data_ptr(), tab.data_ptr(),
                                          max(5, (1 << 30) // sz))
            print(json.dumps({"mem": kind, "kb": sz >> 10, "gb_s": round(sz / dt / 1e9, 2)}))
