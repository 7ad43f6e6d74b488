"""Compressed record batches and old message formats.

The reference consumes through storm-kafka 1.2.3 / kafka-clients 0.11 (pom.xml:40-43,56-58,
76-77), which decode gzip / snappy / lz4 record batches and magic-0/1 message sets
transparently. gale normalises such batches on the consumer thread (csrc/kafka/compress.h) and
routes undecodable ones through --on-error as poison records instead of stalling the source.

Codec parity is pinned three ways: golden bytes written from the format specifications
(snappy raw / xerial framing), the system liblz4 / libzstd loaded through ctypes as independent
encoders and decoders (their shared objects ship in the image; no Python bindings exist), and
Python's zlib / gzip for gzip.
"""

import ctypes
import gzip
import json
import struct
import time

import numpy as np
import pytest

from gale._native import native

C = native()
K = C.kafka

CODECS = ["gzip", "snappy", "lz4"] + (["zstd"] if K.codec_available("zstd") else [])


def _lib(name):
    try:
        return ctypes.CDLL(name)
    except OSError:
        return None


LZ4 = _lib("liblz4.so.1")
ZSTD = _lib("libzstd.so.1")


def payload(n=20000, seed=0):
    """JSON-ish text with repeats (what the input topic carries), plus some noise."""
    rng = np.random.default_rng(seed)
    x = rng.random((1, 8, 8, 3), dtype=np.float32)
    s = C.encode_instances(x) * (1 + n // 2000)
    return s[:n] + bytes(rng.integers(0, 256, 64, dtype=np.uint8))


# ---- snappy: golden streams from the format description ---------------------------------------

def test_snappy_golden_raw_streams():
    # literal "abc", copy-1 (len 9, offset 3), literal "X"
    assert K.decompress("snappy", b"\x0d\x08abc\x15\x03\x00X") == b"abcabcabcabcX"
    # copy-2: 1-byte literal "a", then 63 bytes at offset 1 (run of 'a')
    assert K.decompress("snappy", b"\x40\x00a" + bytes([2 | (62 << 2)]) + b"\x01\x00") == b"a" * 64
    # copy-4: literal "xyz" then 3 bytes at offset 3
    assert K.decompress("snappy", b"\x06\x08xyz" + bytes([3 | (2 << 2)]) + b"\x03\x00\x00\x00") \
        == b"xyzxyz"
    # 60-form literal (length in the next byte): 100 bytes
    body = bytes(range(100))
    assert K.decompress("snappy", b"\x64" + bytes([60 << 2, 99]) + body) == body


def test_snappy_xerial_framing_and_corruption():
    a, b = b"hello " * 50, b"world " * 40
    raw_a, raw_b = K.snappy_compress_raw(a), K.snappy_compress_raw(b)
    framed = (b"\x82SNAPPY\x00" + struct.pack(">ii", 1, 1) + struct.pack(">i", len(raw_a)) + raw_a
              + struct.pack(">i", len(raw_b)) + raw_b)
    assert K.decompress("snappy", framed) == a + b
    with pytest.raises(RuntimeError):
        K.decompress("snappy", b"\x0d\x08abc\x15\x09\x00X")  # offset beyond the output
    with pytest.raises(RuntimeError):
        K.decompress("snappy", framed[:-3])  # truncated block


@pytest.mark.parametrize("n", [0, 1, 3, 17, 1000, 70000, 300000])
def test_snappy_roundtrip_sizes(n):
    d = payload(n)[:n]
    z = K.compress("snappy", d)
    assert z.startswith(b"\x82SNAPPY\x00")  # Kafka's Java client framing
    assert K.decompress("snappy", z) == d
    if n > 2000:
        assert len(z) < len(d)


# ---- lz4: the system liblz4 as the independent codec ------------------------------------------

@pytest.mark.skipif(LZ4 is None, reason="liblz4.so.1 not in this image")
@pytest.mark.parametrize("n", [0, 5, 13, 4096, 65536, 65537, 250000])
def test_lz4_frame_against_system_liblz4(n):
    d = payload(n)[:n]
    # liblz4 -> gale
    LZ4.LZ4F_compressFrameBound.restype = ctypes.c_size_t
    LZ4.LZ4F_compressFrame.restype = ctypes.c_size_t
    LZ4.LZ4F_isError.restype = ctypes.c_uint
    cap = LZ4.LZ4F_compressFrameBound(ctypes.c_size_t(n), None)
    dst = ctypes.create_string_buffer(cap)
    r = LZ4.LZ4F_compressFrame(dst, ctypes.c_size_t(cap), d, ctypes.c_size_t(n), None)
    assert not LZ4.LZ4F_isError(ctypes.c_size_t(r))
    assert K.decompress("lz4", dst.raw[:r]) == d
    # gale -> liblz4 (its frame decoder checks the header checksum: gale's xxh32)
    z = K.compress("lz4", d)
    ctx = ctypes.c_void_p()
    assert LZ4.LZ4F_createDecompressionContext(ctypes.byref(ctx), 100) == 0
    out = ctypes.create_string_buffer(max(1, n))
    dsz, ssz = ctypes.c_size_t(max(1, n)), ctypes.c_size_t(len(z))
    LZ4.LZ4F_decompress.restype = ctypes.c_size_t
    r = LZ4.LZ4F_decompress(ctx, out, ctypes.byref(dsz), z, ctypes.byref(ssz), None)
    LZ4.LZ4F_freeDecompressionContext(ctx)
    assert not LZ4.LZ4F_isError(ctypes.c_size_t(r)) and r == 0  # frame complete
    assert out.raw[:dsz.value] == d and ssz.value == len(z)


def test_xxh32_reference_values():
    # XXH32 test vectors (empty input and "abc", seed 0; the published reference values)
    assert K.xxh32(b"") == 0x02CC5D05
    assert K.xxh32(b"abc") == 0x32D153FF
    assert K.xxh32(b"Nobody inspects the spammish repetition") == 0xE2293B2F


# ---- gzip / zstd ---------------------------------------------------------------------------------

def test_gzip_against_python():
    d = payload(50000)
    assert K.decompress("gzip", gzip.compress(d)) == d
    assert gzip.decompress(K.compress("gzip", d)) == d
    # concatenated members (a valid gzip stream)
    assert K.decompress("gzip", gzip.compress(d[:100]) + gzip.compress(d[100:])) == d


@pytest.mark.skipif(ZSTD is None or not K.codec_available("zstd"), reason="no libzstd")
def test_zstd_against_system_libzstd():
    d = payload(80000)
    ZSTD.ZSTD_compressBound.restype = ctypes.c_size_t
    ZSTD.ZSTD_compress.restype = ctypes.c_size_t
    cap = ZSTD.ZSTD_compressBound(ctypes.c_size_t(len(d)))
    dst = ctypes.create_string_buffer(cap)
    r = ZSTD.ZSTD_compress(dst, ctypes.c_size_t(cap), d, ctypes.c_size_t(len(d)), 5)
    assert K.decompress("zstd", dst.raw[:r]) == d
    z = K.compress("zstd", d)
    ZSTD.ZSTD_decompress.restype = ctypes.c_size_t
    out = ctypes.create_string_buffer(len(d))
    r = ZSTD.ZSTD_decompress(out, ctypes.c_size_t(len(d)), z, ctypes.c_size_t(len(z)))
    assert r == len(d) and out.raw == d


def test_decompression_limit():
    d = b"\x00" * (1 << 20)
    for codec in CODECS:
        with pytest.raises(RuntimeError):
            K.decompress(codec, K.compress(codec, d), limit=1 << 16)


# ---- record batches and message sets ------------------------------------------------------------

def records(n=12, seed=1):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        x = rng.random((1, 4, 4, 3), dtype=np.float32)
        key = None if i % 3 == 0 else f"k{i}".encode()
        out.append((key, C.encode_instances(x), 1000 + i, [("h", b"v")] if i % 4 == 0 else None))
    return out


@pytest.mark.parametrize("codec", CODECS)
def test_compressed_v2_batch_decodes_like_the_plain_one(codec):
    recs = records()
    plain = K.encode_batch(recs, 100, 1000)
    z = K.compress_batch(plain, codec)
    attrs = struct.unpack(">h", z[21:23])[0]
    assert attrs & 7 == ["none", "gzip", "snappy", "lz4", "zstd"].index(codec)
    assert len(z) < len(plain)
    want = K.decode_records(plain, 0, True)
    got = K.decode_records(z, 0, True)
    assert got == want and len(got) == len(recs)
    # a fetch that starts mid-batch skips the records before its offset
    assert [r["offset"] for r in K.decode_records(z, 105, True)] == list(range(105, 112))
    blob, st = K.normalize_records(plain + z, 0, True)
    assert st["converted_batches"] == 1 and st["poison_batches"] == 0
    assert K.decode_records(blob, 0, True) == want + want


@pytest.mark.parametrize("magic", [0, 1])
@pytest.mark.parametrize("codec", ["none", "gzip", "snappy", "lz4"])
def test_legacy_message_sets(magic, codec):
    vals = [f'{{"instances": [[[[{i}.0]]]]}}'.encode() for i in range(7)]
    keys = [None, b"a", None, b"b", None, None, b"c"]
    ms = K.encode_message_set(magic, vals, 40, codec, keys, 123456)
    got = K.decode_records(ms, 0, True)
    assert [r["offset"] for r in got] == list(range(40, 47))
    assert [r["value"] for r in got] == vals and [r["key"] for r in got] == keys
    assert all(r["timestamp"] == (123456 if magic == 1 else -1) for r in got)
    # mid-set fetch position
    assert [r["offset"] for r in K.decode_records(ms, 44, True)] == [44, 45, 46]


def test_poison_batches_become_marked_records():
    recs = records(6)
    good = K.encode_batch(recs, 0, 0)
    # a compressed batch whose payload is garbage but whose CRC32C is valid: decompression fails
    z = bytearray(K.compress_batch(K.encode_batch(recs, 6, 0), "lz4"))
    z[70:90] = b"\xff" * 20
    crc = C.kafka.crc32c(bytes(z[21:])) if hasattr(C.kafka, "crc32c") else None
    if crc is None:
        pytest.skip("no crc32c binding")
    z[17:21] = struct.pack(">I", crc)
    # an unknown codec id (6)
    u = bytearray(K.encode_batch(recs, 12, 0))
    u[22] |= 6
    u[17:21] = struct.pack(">I", C.kafka.crc32c(bytes(u[21:])))
    # a plain batch with a flipped bit (CRC mismatch)
    bad = bytearray(K.encode_batch(recs, 18, 0))
    bad[len(bad) // 2] ^= 1
    tail = K.encode_batch(recs, 24, 0)
    blob = good + bytes(z) + bytes(u) + bytes(bad) + tail
    got = K.decode_records(blob, 0, True)
    assert [r["offset"] for r in got] == list(range(30))
    poison = [r["offset"] for r in got if r.get("poison")]
    assert poison == list(range(6, 24))
    assert all(r["value"] is None for r in got if r.get("poison"))
    _, st = K.normalize_records(blob, 0, True)
    assert st["poison_batches"] == 3 and st["poison_records"] == 18


def test_decompression_budget_is_per_fetch_not_per_batch():
    """the decompression limit bounds the whole normalisation of a partition fetch.
    Five gzip batches of ~20 KB plain each under a 50 KB budget: the blob ends after the batches
    the budget covers (no poison), and normalising again from the next offset - the consumer's
    next fetch - continues where it stopped."""
    recs = [(None, b"0" * 2000, 0, None) for _ in range(10)]
    zs = [K.compress_batch(K.encode_batch(recs, 10 * i, 0), "gzip") for i in range(5)]
    blob_in = b"".join(zs)
    got_all = []
    pos = 0
    calls = 0
    while pos < 50:
        blob, st = K.normalize_records(blob_in, pos, True, limit=50_000)
        assert st["poison_batches"] == 0
        offs = [r["offset"] for r in K.decode_records(blob, 0, True)]
        assert offs and offs[0] == pos and len(offs) <= 30  # <= 2-3 batches per call
        got_all += offs
        pos = offs[-1] + 1
        calls += 1
    assert got_all == list(range(50)) and calls >= 2
    # with the budget spent by earlier batches, a batch over the remaining budget is not poison
    blob, st = K.normalize_records(blob_in, 0, True, limit=30_000)
    assert st["poison_batches"] == 0 and len(K.decode_records(blob, 0, True)) == 10
    # one batch over the whole budget alone is
    _, st = K.normalize_records(zs[0], 0, True, limit=10_000)
    assert st["poison_batches"] == 1


def test_failed_legacy_wrapper_poisons_its_inner_span():
    """a compressed magic-1 wrapper that cannot be decoded covers the offsets after the
    previous entry up to its own (its last inner record's); each becomes a poison record (counted
    in poison_unknown_span, since the inner count itself is unreadable)."""
    vals = [b'{"instances": [[[[1.0]]]]}'] * 4
    first = K.encode_message_set(1, vals, 10, "none")  # offsets 10-13, plain
    bad = bytearray(K.encode_message_set(1, vals, 14, "gzip"))  # wrapper offset 17
    mid = 16 + (len(bad) - 16) // 2
    bad[mid:mid + 6] = b"\xff" * 6  # corrupt the compressed payload ...
    import zlib
    body = bytes(bad[16:])  # ... and fix the message CRC (magic .. value)
    bad[12:16] = struct.pack(">I", zlib.crc32(body))
    _, st = K.normalize_records(first + bytes(bad), 10, True)
    got = K.decode_records(first + bytes(bad), 10, True)
    assert [r["offset"] for r in got] == list(range(10, 18))
    assert [r["offset"] for r in got if r.get("poison")] == [14, 15, 16, 17]
    assert st["poison_records"] == 4 and st["poison_unknown_span"] == 4


# ---- through the broker and the consumer ---------------------------------------------------------

@pytest.fixture()
def broker():
    b = K.Broker()
    b.start()
    b.create_topic("t", 1)
    yield b
    b.stop()


def consume_all(broker, n, check_crcs=True):
    cons = K.Consumer(f"127.0.0.1:{broker.port}", max_wait_ms=50, check_crcs=check_crcs)
    cons.assign("t", [0])
    cons.seek_to("earliest")
    out, t0 = [], time.time()
    while len(out) < n and time.time() - t0 < 20:
        out += cons.poll()
    return out, cons


@pytest.mark.parametrize("codec", CODECS)
def test_producer_compression_roundtrip_through_broker(broker, codec):
    p = K.Producer(f"127.0.0.1:{broker.port}", compression=codec, linger_ms=5,
                   batch_size=1 << 20)
    vals = [payload(3000, seed=i) for i in range(50)]
    for v in vals:
        p.send("t", v, partition=0)
    p.flush()
    p.close()
    out, cons = consume_all(broker, 50)
    assert [r["value"] for r in out] == vals
    assert [r["offset"] for r in out] == list(range(50))
    assert cons.format_stats()["converted_batches"] >= 1
    assert cons.position(0) == 50


@pytest.mark.parametrize("check_crcs", [True, False])
def test_consumer_skips_poison_and_keeps_serving(broker, check_crcs):
    recs = records(5)
    broker.append_batch_repeated("t", 0, K.encode_batch(recs, 0, 0), 1)
    z = bytearray(K.compress_batch(K.encode_batch(recs, 0, 0), "snappy"))
    z[80:100] = b"\x3f" * 20  # invalid snappy element stream
    z[17:21] = struct.pack(">I", C.kafka.crc32c(bytes(z[21:])))
    broker.append_batch_repeated("t", 0, bytes(z), 1)
    broker.append_legacy("t", 0, 1, [b"a", b"b", b"c"], "gzip")
    broker.append_batch_repeated("t", 0, K.compress_batch(K.encode_batch(recs, 0, 0), "lz4"), 1)
    out, cons = consume_all(broker, 18, check_crcs)
    assert [r["offset"] for r in out] == list(range(18))
    assert [r["offset"] for r in out if r.get("poison")] == list(range(5, 10))
    assert [r["value"] for r in out[10:13]] == [b"a", b"b", b"c"]
    st = cons.format_stats()
    assert st["poison_batches"] == 1 and st["poison_records"] == 5
    assert st["converted_batches"] >= 2


def test_unknown_magic_advances_one_record_per_fetch():
    """A batch of a format nothing can read (magic 3) still lets the source move on: its offsets
    run up to the next batch's base offset and come back as poison records; when it is the last
    batch of a fetch, one poison record at the position (so the position advances one per
    fetch). (The embedded broker refuses such a batch on produce, so this runs at the
    records-blob level, as the consumer sees a fetch.)"""
    recs = records(3)
    b = bytearray(K.encode_batch(recs, 0, 0))
    b[16] = 3
    blob = bytes(b) + K.encode_batch(recs, 3, 0)
    seen = [[(r["offset"], bool(r.get("poison"))) for r in K.decode_records(blob, 0, True)]]
    assert seen[0] == [(0, True), (1, True), (2, True), (3, False), (4, False), (5, False)]
    alone = K.decode_records(bytes(b), 1, True)
    assert [(r["offset"], r.get("poison")) for r in alone] == [(1, True)]


# ---- the engine: compressed input served, poison through --on-error ----------------------------

def test_engine_serves_compressed_input_and_routes_poison(broker):
    from gale.config import GaleConfig
    from gale.engine import Engine

    broker.create_topic("in", 1)
    broker.create_topic("out", 1)
    rng = np.random.default_rng(3)
    xs = [rng.random((1, 32, 32, 3), dtype=np.float32) for _ in range(8)]
    enc = [(None, C.encode_instances(x), -1, None) for x in xs]
    broker.append_batch_repeated("in", 0, K.compress_batch(K.encode_batch(enc[:4], 0, 0), "gzip"), 1)
    z = bytearray(K.compress_batch(K.encode_batch(enc[4:6], 0, 0), "lz4"))
    z[75:95] = b"\xee" * 20
    z[17:21] = struct.pack(">I", C.kafka.crc32c(bytes(z[21:])))
    broker.append_batch_repeated("in", 0, bytes(z), 1)
    broker.append_legacy("in", 0, 1, [e[1] for e in enc[6:]], "snappy")
    cfg = GaleConfig(topology_name="c", input_topic="in", output_topic="out",
                     bootstrap=f"127.0.0.1:{broker.port}", start_offset="earliest", stub=True,
                     max_batch=16, max_wait_us=500, on_error="error-json", commit_interval_ms=100)
    eng = Engine(cfg, max_records=8)
    eng.start()
    assert eng.wait(30), eng.stats()
    eng.stop()
    out = broker.read("out", 0)
    vals = [json.loads(r["value"]) for r in out]
    assert sum("predictions" in v for v in vals) == 6
    assert [v["error"] for v in vals if "error" in v] == ["corrupt", "corrupt"]
    st = eng.stats()
    assert st["poison_batches"] == 1 and st["poison_records"] == 2
    assert st["err_corrupt"] == 2 and st["converted_batches"] >= 2


def test_engine_sink_compression(broker):
    """--compression on the sink (kafka-clients compression.type): the output batches are
    compressed on the wire and decode to the same predictions."""
    from gale.config import GaleConfig
    from gale.engine import Engine

    broker.create_topic("in", 1)
    broker.create_topic("out", 1)
    rng = np.random.default_rng(4)
    for _ in range(6):
        broker.append("in", 0, [C.encode_instances(rng.random((1, 32, 32, 3), dtype=np.float32))])
    cfg = GaleConfig(topology_name="z", input_topic="in", output_topic="out",
                     bootstrap=f"127.0.0.1:{broker.port}", start_offset="earliest", stub=True,
                     max_batch=16, max_wait_us=500, compression="lz4")
    eng = Engine(cfg, max_records=6)
    eng.start()
    assert eng.wait(30), eng.stats()
    eng.stop()
    out = broker.read("out", 0)
    assert len(out) == 6 and all(b"predictions" in r["value"] for r in out)
    cons = K.Consumer(f"127.0.0.1:{broker.port}", max_wait_ms=50)
    cons.assign("out", [0])
    cons.seek_to("earliest")
    got = []
    for _ in range(20):
        got += cons.poll()
        if len(got) >= 6:
            break
    assert cons.format_stats()["converted_batches"] >= 1  # it was compressed on the wire


def test_budget_never_stops_before_a_record_past_the_position():
    """the decompression budget may stop a fetch's conversion only once the output
    holds a record at or past the fetch position - the consumer advances from decoded records
    alone, so a stop before any would refetch the same prefix forever. Here the first entry (a
    gzip legacy wrapper, offsets 10-13) lies wholly below the position 14 and is skipped before
    decompression, so the next wrapper gets the budget and the fetch makes progress."""
    vals = [b"7" * 2000] * 4
    below = K.encode_message_set(1, vals, 10, "gzip")   # offsets 10-13
    past = K.encode_message_set(1, vals, 14, "gzip")    # offsets 14-17
    blob, st = K.normalize_records(below + past, 14, True, limit=9000)
    assert [r["offset"] for r in K.decode_records(blob, 0, True)] == [14, 15, 16, 17]
    assert st["poison_batches"] == 0
    # v2: a first batch whose records all lie below the position still lets the next one through
    z0 = K.compress_batch(K.encode_batch([(None, b"1" * 2000, 0, None)] * 4, 0, 0), "gzip")
    z1 = K.compress_batch(K.encode_batch([(None, b"2" * 2000, 0, None)] * 4, 4, 0), "gzip")
    blob, st = K.normalize_records(z0 + z1, 4, True, limit=9000)
    assert [r["offset"] for r in K.decode_records(blob, 0, True)] == [4, 5, 6, 7]
