"""GPU JSON parser throughput (json_count + json_parse kernels) on a batch of InstObj records.

The records are what bench.py streams: uniform [0,1) images in Java Float.toString format
(~35 KB of text per CIFAR image). Reports device time per batch and GB/s of JSON text.
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gale._native import native  # noqa: E402

C = native()
REC = np.dtype([("off", "<i8"), ("len", "<i4"), ("slot", "<i4"), ("images", "<i4"),
                ("status", "<i4"), ("tile0", "<i4"), ("has_cnt", "<i4"), ("cnt_off", "<i8"),
                ("pad", "<i8")])
assert REC.itemsize == C.JSON_RECORD_BYTES, "JsonRecord layout changed (gale/kernels.h)"



def staged_batch(batch, H, W, Cc, distinct=64, seed=0):
    rng = np.random.default_rng(seed)
    texts = []
    for _ in range(min(batch, distinct)):
        rec = C.encode_instances(rng.random((1, H, W, Cc), dtype=np.float32))
        s, off, ln, n = C.scan_instances(rec, H, W, Cc)
        assert s == 0 and n == 1
        texts.append(rec[off:off + ln])
    buf = bytearray()
    recs = np.zeros(batch, dtype=REC)
    tiles = 0
    for i in range(batch):
        t = texts[i % len(texts)]
        recs[i] = (len(buf), len(t), i, 1, 0, tiles, 0, 0, 0)
        tiles += C.json_tile_count(len(buf), len(t))
        buf += t + b" " * ((-len(t)) % 16)
    buf += b" " * 16
    tile_rec = np.zeros(tiles, dtype=np.int32)
    for i, r in enumerate(recs):
        n = C.json_tile_count(int(r["off"]), int(r["len"]))
        tile_rec[r["tile0"]:r["tile0"] + n] = i
    return np.frombuffer(bytes(buf), dtype=np.uint8), recs, tile_rec, tiles


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,64,256,1024")
    ap.add_argument("--shape", default="32,32,3")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    H, W, Cc = (int(v) for v in a.shape.split(","))
    s = torch.cuda.current_stream()
    for b in (int(v) for v in a.batches.split(",")):
        raw, recs, tile_rec, tiles = staged_batch(b, H, W, Cc)
        d_raw = torch.from_numpy(raw.copy()).cuda()
        d_recs0 = torch.from_numpy(recs.view(np.uint8).copy()).cuda()
        d_recs = d_recs0.clone()
        d_tile_rec = torch.from_numpy(tile_rec).cuda()
        d_counts = torch.zeros(tiles, dtype=torch.int32, device="cuda")
        out = torch.empty((b, H, W, Cc), device="cuda")

        def run(count_pass=True):
            C.json_parse_instances(b, tiles, d_recs.data_ptr(), d_tile_rec.data_ptr(),
                                   d_raw.data_ptr(), H, W, Cc, d_counts.data_ptr(),
                                   out.data_ptr(), s.cuda_stream, count_pass)

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        st = d_recs.cpu().numpy().view(REC)["status"]
        assert (st == 0).all(), st
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        # the parse alone, from the counts (the serving step: the ingest pass counted them)
        e0.record()
        for _ in range(a.iters):
            run(False)
        e1.record()
        torch.cuda.synchronize()
        us_parse = e0.elapsed_time(e1) * 1e3 / a.iters
        print(json.dumps(dict(kernel="json_parse_instances", batch=b, tiles=tiles,
                              bytes=int(raw.size), us=round(us, 2), parse_only_us=round(us_parse, 2),
                              gb_s=round(raw.size / us / 1e3, 1),
                              img_s=round(b / us * 1e6))), flush=True)


if __name__ == "__main__":
    main()
