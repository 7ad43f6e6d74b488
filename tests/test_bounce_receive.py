"""The bounce receive (csrc/runtime/pack_tap.h BouncePackTap + csrc/kafka/fetch_framing.h): fetch
bodies pass through a small window; the buffer keeps the nibble-packed text plus a sparse host
copy with only the Kafka framing and the two ends of each value. Checked against a plain
consumer reading the same records: every record's framing (offset, timestamp, key, headers,
value position) decodes identically from the sparse copy, the envelope scan gives the same
array extent, the packed stream expands to the exact value bytes, and the value interiors were
really not written on the host. Windows of 4 KiB to 256 KiB put piece boundaries everywhere."""

import numpy as np
import pytest

from gale._native import native

C = native()
K = C.kafka


@pytest.fixture()
def broker():
    b = K.Broker(max_message_bytes=64 << 20)
    b.start()
    b.create_topic("t", 3)
    yield b
    b.stop()


def fill(b):
    rng = np.random.default_rng(3)
    want = 0
    for i in range(30):
        n = 1 + i % 3
        x = rng.random((n, 32, 32, 3), dtype=np.float32)
        vals = [C.encode_instances(x)]
        keys = [f"key-{i}".encode() * (1 + i % 7)] if i % 2 else None
        b.append("t", i % 3, vals, keys)
        want += 1
    # small values, a null value, a value just over the keep threshold, headers
    b.append("t", 0, [b'{"instances": [[[[1.0]]]]}', None, b"x" * 400], None)
    hdr_batch = K.encode_batch([(b"hk", b'{"instances":' + b"[" * 50 + b"]" * 50 + b"}", -1,
                                 [("h1", b"v" * 300), ("h2", None)])], 0, 0)
    b.append_batch_repeated("t", 1, hdr_batch, 2)
    # a compressed batch and an old-format message set (the consumer restores and normalises)
    b.append_batch_repeated("t", 2, K.compress_batch(
        K.encode_batch([(None, C.encode_instances(rng.random((1, 32, 32, 3),
                                                            dtype=np.float32)), -1, None)], 0, 0),
        "lz4"), 1)
    b.append_legacy("t", 2, 1, [b'{"instances": [[[[2.0]]]]}'], "gzip")
    return want + 3 + 2 + 1 + 1


def consume(b, n, **kw):
    cons = K.Consumer(f"127.0.0.1:{b.port}", max_wait_ms=20, fetch_max_bytes=1 << 20,
                      partition_max_bytes=600 << 10, **kw)
    cons.assign("t", [0, 1, 2])
    cons.seek_to("earliest")
    out = []
    for _ in range(400):
        got = cons.poll_bodies() if kw.get("bounce_pack") else cons.poll()
        out += got
        if sum(len(f["records"]) for f in out) >= n if kw.get("bounce_pack") else len(out) >= n:
            break
    return out


@pytest.mark.parametrize("window_kb", [4, 37, 256])
def test_bounce_receive_matches_plain_consumer(broker, window_kb):
    n = fill(broker)
    plain = {(r["partition"], r["offset"]): r for r in consume(broker, n)}
    assert len(plain) == n
    fetches = consume(broker, n, bounce_pack=True, bounce_window_kb=window_kb)
    seen, skipped_any = 0, False
    for f in fetches:
        host, full = f["host"], f.get("unpacked")
        for r in f["records"]:
            p = plain[(r["partition"], r["offset"])]
            seen += 1
            assert r["timestamp"] == p["timestamp"] and r["key"] == p["key"]
            assert r["headers"] == p["headers"]
            v = p["value"]
            if v is None:
                assert r["value_len"] == -1
                continue
            assert r["value_len"] == len(v)
            lo, hi = r["value_off"], r["value_off"] + len(v)
            body = full if f["sparse"] else host
            assert body[lo:hi] == v  # the text, exactly (expanded from the packed stream)
            if f["sparse"]:
                # the envelope scan on the sparse copy sees the same array extent
                st, off, ln = r["scan"]
                if v.lstrip().startswith(b'{"instances"') and v.rstrip().endswith(b"]}"):
                    assert st == 0 and v[off] == ord("[") and v[off + ln - 1] == ord("]")
                # the ends are on the host, a large value's interior is not
                k = min(200, len(v))
                assert host[lo:lo + k] == v[:k] and host[hi - min(50, len(v)):hi] == v[-50:]
                if len(v) > 10000 and host[lo + 300:hi - 100] != v[300:-100]:
                    skipped_any = True
    assert seen == n
    assert skipped_any, "no value interior was skipped on the host"
    assert any(f["sparse"] for f in fetches)
    assert all(f["packed_bytes"] < 0.6 * f["size"] for f in fetches if f["sparse"])
