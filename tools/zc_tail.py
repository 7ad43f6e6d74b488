"""Fetch latency of one stored batch (>= 64 KiB, so the zero-copy broker splices it) over
loopback, copying vs zero-copy broker: a fetch response whose last piece was spliced with
SPLICE_F_MORE held its sub-MSS tail segment until a later ACK (tens of ms) - see
Broker::splice_chunk. Prints p50 / p99 / max per mode."""
import os
import sys
import time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gale._native import native
C = native(); K = C.kafka
for zc in (False, True):
    b = K.Broker(zero_copy=zc); b.start(); b.create_topic("in", 1)
    x = np.random.default_rng(0).random((8, 32, 32, 3), dtype=np.float32)
    doc = C.encode_instances(x)  # ~280 KB: one stored batch >= 64 KiB -> spliced
    b.append("in", 0, [doc])
    c = K.Consumer(f"127.0.0.1:{b.port}", max_wait_ms=20, auto_offset_reset="earliest")
    c.assign("in", [0])
    ts = []
    for i in range(200):
        c.seek(0, 0)
        t0 = time.perf_counter()
        fs = c.poll()
        while not fs:
            fs = c.poll()
        ts.append(time.perf_counter() - t0)
    ts = np.array(ts) * 1e3
    print("zc", zc, "p50 %.3f p99 %.3f max %.3f ms" % (np.percentile(ts, 50), np.percentile(ts, 99), ts.max()))
    b.stop()
