"""Kafka wire protocol: golden bytes built independently with ``struct`` from the protocol spec
(RecordBatch v2, request header v1, Metadata v4 / Fetch v4 / Produce v3 / ListOffsets v1 /
OffsetCommit v2 requests), CRC32C and Java-compatible murmur2 partitioning."""

import struct

import pytest

from gale._native import native

K = native().kafka


def kstr(s: str) -> bytes:
    b = s.encode()
    return struct.pack(">h", len(b)) + b


def zigzag(v: int) -> bytes:
    u = (v << 1) ^ (v >> 63)
    u &= (1 << 64) - 1
    out = bytearray()
    while u >= 0x80:
        out.append((u & 0x7F) | 0x80)
        u >>= 7
    out.append(u)
    return bytes(out)


def _crc_table():
    t = []
    for n in range(256):
        c = n
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
        t.append(c)
    return t


_CRC_T = _crc_table()


def crc32c_ref(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc = (crc >> 8) ^ _CRC_T[(crc ^ b) & 0xFF]
    return crc ^ 0xFFFFFFFF


def test_crc32c_vectors():
    assert K.crc32c(b"123456789") == 0xE3069283  # the standard CRC-32C check value
    assert K.crc32c(b"") == 0
    data = bytes(range(256)) * 37 + b"tail"
    assert K.crc32c(data) == crc32c_ref(data)
    assert K.crc32c(data[3:]) == crc32c_ref(data[3:])  # unaligned start


def test_crc32c_all_paths_lengths_and_offsets():
    """Every length class of the dispatch (bytewise head, VPCLMULQDQ 256-B folding loop and its
    64-B tail loop, 3-stream crc32q blocks, 8-B and 1-B tails) at several alignments."""
    import random

    rng = random.Random(7)
    buf = bytes(rng.getrandbits(8) for _ in range(70000))
    lengths = list(range(0, 70)) + [255, 256, 257, 319, 320, 321, 511, 512, 575, 1000, 4096,
                                     8191, 24576 + 17, 65536 + 3]
    for n in lengths:
        for off in (0, 1, 5, 13):
            d = buf[off:off + n]
            assert K.crc32c(d) == crc32c_ref(d), (n, off)


@pytest.mark.parametrize("key,expected", [
    (b"21", -973932308), (b"foobar", -790332482), (b"a-little-bit-long-string", -985981536),
    (b"a-little-bit-longer-string", -1486304829),
    (b"lkjh234lh9fiuh90y23oiuhsafujhadof229phr9h19h89h8", -58897971), (b"abc", 479470107),
])
def test_murmur2_matches_java_kafka(key, expected):
    # values from Apache Kafka's UtilsTest.testMurmur2 (DefaultPartitioner compatibility)
    assert K.murmur2(key) == expected


def record_v2(offset_delta: int, ts_delta: int, key, value, headers=()) -> bytes:
    body = bytearray(b"\x00")  # attributes
    body += zigzag(ts_delta) + zigzag(offset_delta)
    body += zigzag(-1) if key is None else zigzag(len(key)) + key
    body += zigzag(-1) if value is None else zigzag(len(value)) + value
    body += zigzag(len(headers))
    for hk, hv in headers:
        body += zigzag(len(hk)) + hk + (zigzag(-1) if hv is None else zigzag(len(hv)) + hv)
    return zigzag(len(body)) + bytes(body)


def batch_v2(base_offset, base_ts, records, max_ts=None) -> bytes:
    recs = b"".join(records)
    after_crc = struct.pack(">hiqqqhii", 0, len(records) - 1, base_ts,
                            base_ts if max_ts is None else max_ts, -1, -1, -1, len(records)) + recs
    crc = crc32c_ref(after_crc)
    after_len = struct.pack(">ibI", -1, 2, crc) + after_crc
    return struct.pack(">qi", base_offset, len(after_len)) + after_len


def test_record_batch_golden_bytes():
    recs = [(None, b"hello", 1000, None), (b"k", None, 1005, [("h", b"v"), ("n", None)])]
    got = K.encode_batch(recs, 7, 1000)
    exp = batch_v2(7, 1000, [record_v2(0, 0, None, b"hello"),
                             record_v2(1, 5, b"k", None, [(b"h", b"v"), (b"n", None)])],
                   max_ts=1005)
    assert got == exp
    dec = K.decode_records(got, 0, True)
    assert [(r["offset"], r["timestamp"], r["key"], r["value"]) for r in dec] == [
        (7, 1000, None, b"hello"), (8, 1005, b"k", None)]
    assert dec[1]["headers"] == [("h", b"v"), ("n", None)]


def test_decode_skips_records_before_fetch_offset_and_partial_tail():
    b1 = K.encode_batch([(None, b"a", -1, None), (None, b"b", -1, None)], 10, 0)
    b2 = K.encode_batch([(None, b"c", -1, None)], 12, 0)
    blob = b1 + b2 + b2[:20]  # a truncated trailing batch is legal in a Fetch response
    dec = K.decode_records(blob, 11, True)
    assert [(r["offset"], r["value"]) for r in dec] == [(11, b"b"), (12, b"c")]


def test_decode_detects_corruption():
    b = bytearray(K.encode_batch([(None, b"payload", -1, None)], 0, 0))
    b[-3] ^= 0xFF
    # a corrupt batch never raises out of the consumer (that would stall the source): its
    # records come back as poison markers for the error policy (csrc/kafka/compress.h)
    (r,) = K.decode_records(bytes(b), 0, True)
    assert r["poison"] and r["value"] is None and r["offset"] == 0
    (r,) = K.decode_records(bytes(b), 0, False)  # check_crcs=False skips validation
    assert not r.get("poison") and r["value"] is not None


def test_request_header_golden():
    got = K.encode("request_header", dict(api_key=1, api_version=4, correlation_id=42,
                                          client_id="gale"))
    assert got == struct.pack(">hhi", 1, 4, 42) + kstr("gale")


def test_metadata_request_v4_golden():
    got = K.encode("metadata_request", dict(topics=["in", "out"], allow_auto_topic_creation=True))
    assert got == struct.pack(">i", 2) + kstr("in") + kstr("out") + b"\x01"
    got_all = K.encode("metadata_request", dict(topics=None, allow_auto_topic_creation=False))
    assert got_all == struct.pack(">i", -1) + b"\x00"


def test_fetch_request_v4_golden():
    got = K.encode("fetch_request", dict(max_wait_ms=100, min_bytes=1, max_bytes=1 << 20,
                                         topic="in", partitions=[(0, 5, 4096), (3, 0, 1024)]))
    exp = struct.pack(">iiiib", -1, 100, 1, 1 << 20, 0) + struct.pack(">i", 1) + kstr("in")
    exp += struct.pack(">i", 2) + struct.pack(">iqi", 0, 5, 4096) + struct.pack(">iqi", 3, 0, 1024)
    assert got == exp


def test_produce_request_v3_golden():
    batch = K.encode_batch([(None, b"x", -1, None)], 0, 0)
    got = K.encode("produce_request", dict(acks=-1, timeout_ms=1500, topic="out", partition=2,
                                           records=batch))
    exp = struct.pack(">hhi", -1, -1, 1500) + struct.pack(">i", 1) + kstr("out")
    exp += struct.pack(">i", 1) + struct.pack(">ii", 2, len(batch)) + batch
    assert got == exp


def test_list_offsets_and_offset_commit_golden():
    got = K.encode("list_offsets_request", dict(topic="in", partition=1, timestamp=-2))
    assert got == struct.pack(">ii", -1, 1) + kstr("in") + struct.pack(">iiq", 1, 1, -2)
    got = K.encode("offset_commit_request", dict(group_id="g", topic="in", partition=0,
                                                 offset=99))
    exp = kstr("g") + struct.pack(">i", -1) + kstr("") + struct.pack(">q", -1)
    exp += struct.pack(">i", 1) + kstr("in") + struct.pack(">iiq", 1, 0, 99) + kstr("")
    assert got == exp


def test_versions_table():
    # one version per API, all still served by Kafka 4.x (KIP-896)
    assert [K.api_version(k) for k in (0, 1, 2, 3, 8, 9, 10, 18, 19)] == [3, 4, 1, 4, 2, 1, 1, 0, 2]
