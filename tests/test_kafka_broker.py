"""Embedded broker <-> native client integration (the LocalCluster / embedded-Kafka role,
SURVEY.md §4), plus a raw-socket client written here in Python so the broker is also checked
against an implementation that shares no code with it."""

import socket
import struct
import threading
import time

import pytest

from gale._native import native

K = native().kafka


@pytest.fixture()
def broker():
    b = K.Broker(default_partitions=3)
    b.start()
    yield b
    b.stop()


def bs(b):
    return f"127.0.0.1:{b.port}"


def raw_request(port, api_key, version, body, corr=7):
    s = socket.create_connection(("127.0.0.1", port))
    hdr = struct.pack(">hhi", api_key, version, corr) + struct.pack(">h", 3) + b"raw"
    msg = hdr + body
    s.sendall(struct.pack(">i", len(msg)) + msg)
    size = struct.unpack(">i", s.recv(4, socket.MSG_WAITALL))[0]
    data = b""
    while len(data) < size:
        data += s.recv(size - len(data))
    s.close()
    assert struct.unpack(">i", data[:4])[0] == corr
    return data[4:]


def test_raw_socket_api_versions_and_metadata(broker):
    resp = raw_request(broker.port, 18, 0, b"")
    err, n = struct.unpack(">hi", resp[:6])
    assert err == 0
    apis = {struct.unpack(">hhh", resp[6 + 6 * i:12 + 6 * i])[0]: struct.unpack(
        ">hhh", resp[6 + 6 * i:12 + 6 * i])[1:] for i in range(n)}
    assert apis[1] == (4, 4) and apis[0] == (3, 3) and apis[3] == (4, 4)
    # a flexible ApiVersions (v3) gets UNSUPPORTED_VERSION in the v0 format, like Kafka
    assert struct.unpack(">h", raw_request(broker.port, 18, 3, b"")[:2])[0] == 35
    body = struct.pack(">i", 1) + struct.pack(">h", 5) + b"topic" + b"\x01"
    d = K.decode("metadata_response", raw_request(broker.port, 3, 4, body))
    assert d["brokers"] == [(0, "127.0.0.1", broker.port)]
    err, parts = d["topics"]["topic"]
    assert err == 0 and len(parts) == 3 and all(p[1] == 0 for p in parts)  # auto-created


def test_produce_consume_roundtrip(broker):
    p = K.Producer(bs(broker), acks=1)
    acks = []
    for i in range(30):
        p.send("t", f"v{i}".encode(), key=None if i % 2 else f"k{i}".encode(),
               headers=[("h", b"x")] if i == 0 else None,
               callback=lambda e, part, off: acks.append((e, part, off)))
    p.flush()
    assert len(acks) == 30 and all(a[0] == 0 for a in acks)
    c = K.Consumer(bs(broker), auto_offset_reset="earliest")
    c.assign("t", [])
    c.seek_to("earliest")
    got = []
    for _ in range(20):
        got += c.poll()
        if len(got) >= 30:
            break
    assert sorted(r["value"] for r in got) == sorted(f"v{i}".encode() for i in range(30))
    assert next(r for r in got if r["value"] == b"v0")["headers"] == [("h", b"x")]
    # keyed records follow Java's murmur2 partitioner
    parts = {r["value"]: r["partition"] for r in got}
    for i in range(0, 30, 2):
        assert parts[f"v{i}".encode()] == (K.murmur2(f"k{i}".encode()) & 0x7FFFFFFF) % 3
    p.close()


def test_long_poll_fetch_wakes_on_produce(broker):
    broker.create_topic("lp", 1)
    c = K.Consumer(bs(broker), max_wait_ms=3000)
    c.assign("lp", [0])
    c.seek_to("latest")
    out = {}

    def consume():
        t = time.perf_counter()
        out["recs"] = c.poll()
        out["dt"] = time.perf_counter() - t

    th = threading.Thread(target=consume)
    th.start()
    time.sleep(0.2)
    broker.append("lp", 0, [b"wake"])
    th.join()
    assert [r["value"] for r in out["recs"]] == [b"wake"]
    assert out["dt"] < 2.0  # answered by the append, not by max_wait_ms


def test_offsets_latest_earliest_committed(broker):
    broker.create_topic("o", 1)
    for i in range(10):
        broker.append("o", 0, [str(i).encode()])
    c = K.Consumer(bs(broker), group_id="grp", auto_offset_reset="earliest")
    c.assign("o", [0])
    c.seek_to("latest")
    assert c.position(0) == 10
    c.seek_to("earliest")
    assert c.position(0) == 0
    c.seek_to("committed")  # nothing committed -> auto_offset_reset
    assert c.position(0) == 0
    c.commit({0: 6})
    assert c.committed(0) == 6 and broker.committed("grp", "o", 0) == 6
    c2 = K.Consumer(bs(broker), group_id="grp")
    c2.assign("o", [0])
    c2.seek_to("committed")
    assert [r["value"] for r in c2.poll()] == [b"6", b"7", b"8", b"9"]


def test_acks_zero_and_null_values(broker):
    p = K.Producer(bs(broker), acks=0)
    p.send("z", None, partition=0)
    p.send("z", b"x", partition=0)
    p.flush()
    time.sleep(0.2)
    recs = broker.read("z", 0)
    assert [r["value"] for r in recs] == [None, b"x"]
    p.close()


def test_message_too_large_is_rejected():
    b = K.Broker(max_message_bytes=1000)
    b.start()
    try:
        p = K.Producer(bs(b))
        errs = []
        p.send("big", b"x" * 5000, partition=0, callback=lambda e, pa, o: errs.append(e))
        p.flush()  # separate batches: the broker rejects a whole batch
        p.send("big", b"small", partition=0, callback=lambda e, pa, o: errs.append(e))
        p.flush()
        assert sorted(errs) == [0, 10]  # MESSAGE_TOO_LARGE for the big batch only
        p.close()
    finally:
        b.stop()


def test_retention_drops_old_segments():
    b = K.Broker(retention_bytes=2000)
    b.start()
    try:
        b.create_topic("r", 1)
        for i in range(50):
            b.append("r", 0, [b"y" * 100])
        assert b.log_end("r", 0) == 50
        assert 0 < b.log_start("r", 0) < 50
        c = K.Consumer(bs(b), auto_offset_reset="earliest")
        c.assign("r", [0])
        c.seek(0, 0)  # out of range -> reset to earliest retained, records on the next poll
        recs = c.poll() or c.poll()
        assert recs and recs[0]["offset"] == b.log_start("r", 0)
    finally:
        b.stop()


def test_multi_broker_cluster_leadership():
    b0 = K.Broker(node_id=0)
    b1 = K.Broker(node_id=1)
    b0.start()
    b1.start()
    try:
        nodes = [(0, "127.0.0.1", b0.port), (1, "127.0.0.1", b1.port)]
        for b in (b0, b1):
            b.set_cluster(nodes)
            b.create_topic("m", 4)
        assert b0.leads(0) and b1.leads(1) and not b0.leads(1)
        p = K.Producer(bs(b0))  # bootstrap via node 0 only
        for i in range(8):
            p.send("m", f"{i}".encode(), partition=i % 4)
        p.flush()
        assert b0.log_end("m", 0) == 2 and b1.log_end("m", 1) == 2
        assert b0.log_end("m", 1) == 0  # node 0 does not host partition 1's log
        c = K.Consumer(bs(b1), auto_offset_reset="earliest")
        c.assign("m", [])
        c.seek_to("earliest")
        got = []
        for _ in range(10):
            got += c.poll()
            if len(got) == 8:
                break
        assert sorted(int(r["value"]) for r in got) == list(range(8))
        p.close()
    finally:
        b0.stop()
        b1.stop()


def test_broker_stats_and_topic_management(broker):
    assert broker.create_topic("a", 2) is True
    assert broker.create_topic("a", 2) is False
    assert broker.partitions("a") == 2 and broker.partitions("nope") == -1
    with pytest.raises(ValueError):
        broker.create_topic("bad topic!", 1)
    s = broker.stats()
    assert set(s) >= {"requests", "bytes_in", "bytes_out", "records_in"}


def test_zero_copy_fetch_is_byte_identical():
    """zero_copy=True: stored batches >= 64 KiB go out with vmsplice/splice (headers and small
    pieces by writev, interleaved in order). The consumer sees exactly the bytes of the
    writev path, CRC-checked, across many partitions and fetches."""
    import numpy as np

    rng = np.random.default_rng(3)
    vals = [rng.integers(0, 256, size=int(n), dtype=np.uint8).tobytes()
            for n in rng.integers(1000, 300_000, size=60)]
    got = {}
    for zc in (False, True):
        b = K.Broker(zero_copy=zc)
        b.start()
        b.create_topic("z", 3)
        for i in range(0, len(vals), 4):
            b.append("z", (i // 4) % 3, vals[i:i + 4])
        c = K.Consumer(bs(b), auto_offset_reset="earliest", check_crcs=True,
                       partition_max_bytes=1 << 20)
        c.assign("z", [])
        c.seek_to("earliest")
        recs = []
        for _ in range(200):
            recs += c.poll()
            if len(recs) >= len(vals):
                break
        got[zc] = sorted((r["partition"], r["offset"], r["value"]) for r in recs)
        spliced = b.stats()["bytes_spliced"]
        assert (spliced > 0) == zc
        b.stop()
    assert len(got[True]) == len(vals) and got[True] == got[False]


def test_log_append_time_stamps_shared_batches_with_valid_crc():
    """LogAppendTime: the broker stamps each appended batch (attributes bit 3 + maxTimestamp) and
    patches its CRC32C without re-reading the batch; one shared batch appended twice carries two
    different stamps, every fetched batch passes the consumer's CRC check and each record reports
    the append time."""
    import numpy as np

    imgs = np.random.default_rng(0).random((8, 4, 4, 3), dtype=np.float32)
    bset = K.synthetic_batches(imgs, 1, 4, 2, "id-")
    assert len(bset) == 2 and bset.records == 8
    b = K.Broker(log_append_time=True)
    b.start()
    try:
        b.create_topic("t", 1)
        t0 = int(time.time() * 1000)
        b.append_cycled("t", 0, bset, 2, 0)
        time.sleep(0.02)
        b.append_cycled("t", 0, bset, 2, 0)  # the same two blobs again, later
        t1 = int(time.time() * 1000)
        c = K.Consumer(bs(b))
        c.assign("t", [0])
        c.seek_to("earliest")
        got = []
        for _ in range(20):
            got += c.poll()
            if len(got) >= 16:
                break
        assert len(got) == 16
        ts = [r["timestamp"] for r in got]
        assert all(t0 <= t <= t1 for t in ts)
        assert ts[0] < ts[-1]  # second append stamped later
        assert [r["key"] for r in got[:8]] == [f"id-{i}".encode() for i in range(8)]
        # the stored blob itself is untouched: the stamp lives in the broker's segment
        assert K.decode_records(bset.batch(0), 0, True)[0]["timestamp"] == 0
    finally:
        b.stop()


def test_crc32c_combine_and_shift():
    import os as _os

    a, bb = _os.urandom(1000), _os.urandom(3333)
    ca, cb = K.crc32c(a), K.crc32c(bb)
    assert K.crc32c_combine(ca, cb, len(bb)) == K.crc32c(a + bb)


def test_producer_backlog_leaves_in_request_sized_batches(broker):
    """Records that pile up behind a busy sender are drained in batches of at most
    max_request_size (at least one record each), not as one batch of the whole backlog; order
    within the partition is kept and every record is acknowledged once."""
    p = K.Producer(bs(broker), acks=1, max_request_size=4096, max_in_flight=2)
    acks = []
    n = 400
    for i in range(n):
        p.send("big", (b"%04d" % i) * 50, partition=0,
               callback=lambda e, part, off: acks.append((e, off)))
    p.flush()
    assert len(acks) == n and all(e == 0 for e, _ in acks)
    assert sorted(off for _, off in acks) == list(range(n))
    st = p.stats()
    assert st["requests"] >= n * 200 // 4096  # 200-byte values: ~20 per 4 KB request
    c = K.Consumer(bs(broker), auto_offset_reset="earliest")
    c.assign("big", [0])
    c.seek_to("earliest")
    got = []
    for _ in range(50):
        got += c.poll()
        if len(got) >= n:
            break
    assert [r["value"][:4] for r in got] == [b"%04d" % i for i in range(n)]


def test_producer_chunks_with_headers_fit_max_request_size():
    """The producer cuts a backlog into batches by an upper bound of each record's encoded size
    that includes its headers (the __TypeId__ header of --type-id-header adds ~28 bytes to a
    ~120-byte prediction record): every batch stays within max_request_size, so a broker whose
    message.max.bytes equals it accepts them all."""
    cap = 16 << 10
    b = K.Broker(max_message_bytes=cap)
    b.start()
    try:
        b.create_topic("h", 1)
        p = K.Producer(bs(b), linger_ms=300, batch_size=1 << 20, max_request_size=cap)
        errs = []
        n = 2000
        for i in range(n):
            p.send("h", b"x" * 120, partition=0, headers=[("__TypeId__", b"java.lang.String")],
                   callback=lambda e, pa, o: errs.append(e))
        p.flush()
        assert len(errs) == n and set(errs) == {0}
        assert p.stats()["requests"] >= n * 150 // cap
        p.close()
    finally:
        b.stop()
