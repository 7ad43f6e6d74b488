"""Device throughput of the GPU ingest kernels on their own (no other stream competing): the fused
CRC32C + token-count pass (ingest_crc_count) over a fetch-sized buffer and the JSON parse of its
records, for CIFAR (32x32x3, ~35 KB per image) and ImageNet (224x224x3, ~1.7 MB) records.

usage: python tools/bench_ingest.py [--iters 50]
Prints one JSON line per (shape, kernel): us per launch and GB/s of JSON text.
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
K = C.kafka
REC = np.dtype([("off", "<i8"), ("len", "<i4"), ("slot", "<i4"), ("images", "<i4"),
                ("status", "<i4"), ("tile0", "<i4"), ("has_cnt", "<i4"), ("cnt_off", "<i8"),
                ("pad", "<i8")])


def build(shape, nrec, seed=0):
    rng = np.random.default_rng(seed)
    H, W, Cc = shape
    x = rng.random((1, H, W, Cc), dtype=np.float32)
    s, off, ln, n = C.scan_instances(C.encode_instances(x), H, W, Cc)
    txt = C.encode_instances(x)[off:off + ln]
    buf = bytearray()
    recs = np.zeros(nrec, dtype=REC)
    tiles = 0
    for i in range(nrec):
        recs[i] = (len(buf), len(txt), i, 1, 0, tiles, 0, 0, 0)
        tiles += C.json_tile_count(len(buf), len(txt))
        buf += txt + b" " * ((-len(txt)) % 16)
    buf += b" " * 64
    tile_rec = np.zeros(tiles, dtype=np.int32)
    groups = []
    for i, r in enumerate(recs):
        t = C.json_tile_count(int(r["off"]), int(r["len"]))
        tile_rec[r["tile0"]:r["tile0"] + t] = i
        recs[i]["pad"] = len(groups)  # JsonRecord::grp0
        groups += [(i, t0) for t0 in range(0, t, C.GROUP_TILES)]
    n = len(buf) - 64
    wins = [(n - 4096 * k, 4096) for k in range(n // 4096)][::-1]
    if n % 4096:
        wins = [(n - 4096 * len(wins), n % 4096)] + wins
    ch = np.zeros(len(wins), dtype=[("end", "<i8"), ("len", "<i4"), ("pad", "<i4")])
    for i, (e, w) in enumerate(wins):
        ch[i] = (e, w, 0)
    return bytes(buf), recs, tile_rec, tiles, ch, n, np.array(groups, dtype=np.int32)


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    s = torch.cuda.current_stream().cuda_stream
    tables = torch.tensor(np.array(K.crc32c_device_tables(), dtype=np.uint32).view(np.int32),
                          device="cuda")
    for name, shape, nrec in (("cifar_fetch", (32, 32, 3), 64), ("cifar_batch", (32, 32, 3), 256),
                              ("imagenet_fetch", (224, 224, 3), 9),
                              ("imagenet_batch", (224, 224, 3), 256)):
        buf, recs, tile_rec, tiles, ch, n, groups = build(shape, nrec)
        dgrp = torch.from_numpy(groups.reshape(-1)).cuda()
        d = torch.frombuffer(bytearray(buf), dtype=torch.uint8).cuda()
        dch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
        dmap = torch.from_numpy(tile_rec).cuda()
        drec = torch.from_numpy(recs.view(np.uint8).copy()).cuda()
        crc = torch.zeros(len(ch), dtype=torch.int32, device="cuda")
        cnt = torch.zeros(tiles + len(groups), dtype=torch.int32, device="cuda")
        cnt_p = torch.zeros(tiles, dtype=torch.int32, device="cuda")  # the parse's own pass
        gsum = torch.zeros(max(1, len(groups)), dtype=torch.int32, device="cuda")
        H, W, Cc = shape
        out = torch.empty((nrec, H, W, Cc), device="cuda")

        def ingest():
            C.ingest_crc_count(d.data_ptr(), dch.data_ptr(), len(ch), tables.data_ptr(),
                               crc.data_ptr(), nrec, len(groups), drec.data_ptr(),
                               dgrp.data_ptr(), cnt.data_ptr(), gsum.data_ptr(), s)

        packed, tab = C.text_pack(buf[:n])
        dp = torch.frombuffer(bytearray(packed + bytes(64)), dtype=torch.uint8).cuda()
        dt = torch.from_numpy(tab.astype(np.int64)).to(torch.int32).cuda()
        text = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        gbad = torch.zeros(max(1, len(groups)), dtype=torch.int32, device="cuda")

        def ingest_packed():  # the engine's form: the packed body, expansion folded in
            C.ingest_crc_count(d.data_ptr(), dch.data_ptr(), len(ch), tables.data_ptr(),
                               crc.data_ptr(), nrec, len(groups), drec.data_ptr(),
                               dgrp.data_ptr(), cnt.data_ptr(), gsum.data_ptr(), s,
                               gbad=gbad.data_ptr(), packed=dp.data_ptr(), tab=dt.data_ptr(),
                               text_out=text.data_ptr())

        def unpack_then_ingest():  # round 4: text_unpack pass, then crc+count on the text
            C.text_unpack(dp.data_ptr(), dt.data_ptr(), n, text.data_ptr(), s)
            C.ingest_crc_count(text.data_ptr(), dch.data_ptr(), len(ch), tables.data_ptr(),
                               crc.data_ptr(), nrec, len(groups), drec.data_ptr(),
                               dgrp.data_ptr(), cnt.data_ptr(), gsum.data_ptr(), s)

        def crc_only():
            C.ingest_crc_count(d.data_ptr(), dch.data_ptr(), len(ch), tables.data_ptr(),
                               crc.data_ptr(), 0, 0, drec.data_ptr(), dgrp.data_ptr(),
                               cnt.data_ptr(), gsum.data_ptr(), s)

        def parse():
            C.json_parse_instances(nrec, tiles, drec.data_ptr(), dmap.data_ptr(), d.data_ptr(), H,
                                   W, Cc, cnt_p.data_ptr(), out.data_ptr(), s, count_pass=True)

        # the replica's parse of ingested records: the ingest pass's count blocks, no count pass
        ingest()
        recs2 = recs.copy()
        recs2["has_cnt"] = 1
        recs2["cnt_off"] = [cnt.data_ptr() + 4 * (int(r["tile0"]) + int(r["pad"])) - d.data_ptr()
                            for r in recs]
        drec2 = torch.from_numpy(recs2.view(np.uint8).copy()).cuda()

        def parse_cnt():
            C.json_parse_instances(nrec, tiles, drec2.data_ptr(), dmap.data_ptr(), d.data_ptr(),
                                   H, W, Cc, cnt_p.data_ptr(), out.data_ptr(), s,
                                   count_pass=False)

        for kname, fn in (("crc+count", ingest), ("crc", crc_only),
                          ("crc+count+expand(packed)", ingest_packed),
                          ("unpack;crc+count (r4)", unpack_then_ingest),
                          ("count+parse", parse), ("parse(ingest counts)", parse_cnt)):
            us = timed(fn, a.iters)
            print(json.dumps(dict(case=name, kernel=kname, records=nrec, text_mb=round(n / 1e6, 2),
                                  us=round(us, 1), gb_s=round(n / us / 1e3, 1))), flush=True)
        for dr in (drec, drec2):
            st = dr.cpu().numpy().view(REC)["status"]
            assert (st == 0).all(), st


if __name__ == "__main__":
    main()
