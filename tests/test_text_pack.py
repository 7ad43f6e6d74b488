"""Nibble transport for the host -> GPU link (csrc/codec/text_pack.h): lossless round trips of
Jackson InstObj text, Kafka framing and arbitrary bytes, the vector packer against the scalar
reference, and the device expansion (text_unpack in csrc/kernels/ingest.hip) against the host
reference."""

import numpy as np
import pytest

from gale._native import native

N = native()


def _jackson_text(n_img=2, seed=0):
    x = np.random.default_rng(seed).random((n_img, 32, 32, 3), dtype=np.float32)
    x[0, 0, 0, :] = [1e-5, -3.5e-7, 12345678.0]  # exponent forms and a minus sign
    return N.encode_instances(x)


def _cases():
    rng = np.random.default_rng(1)
    doc = _jackson_text()
    yield "empty", b""
    yield "short", b"[0.5,1.0]"
    yield "one_block", (b"0.123456789," * 6)[:64]
    yield "instobj", doc
    yield "instobj_tail", doc[:-17]
    yield "framing", b"\x00\x00\x01\x02" * 40 + doc + b"\x7f\x80\xff" * 50 + doc[:1000]
    yield "random", rng.integers(0, 256, 10000, dtype=np.uint8).tobytes()
    # alphabet-only bytes in random order (every code in every nibble position)
    alpha = np.frombuffer(b"0123456789[],-.E", np.uint8)
    yield "alphabet", alpha[rng.integers(0, 16, 4096 * 3 + 5)].tobytes()
    # a block that differs from the alphabet in its last byte only
    yield "edge", b"1" * 63 + b"e" + b"2" * 64 + b"\xb0" * 64 + b"3" * 64


@pytest.mark.parametrize("name,data", list(_cases()))
@pytest.mark.parametrize("scalar", [True, False])
def test_round_trip(name, data, scalar):
    if not scalar and not N.text_pack_fast():
        pytest.skip("no AVX-512 VBMI on this host")
    packed, tab = N.text_pack(data, scalar)
    assert len(tab) == 2 * (-(-len(data) // 2048))
    assert N.text_unpack_host(packed, tab, len(data)) == data
    if not scalar:
        p2, t2 = N.text_pack(data, True)
        assert packed == p2 and np.array_equal(tab, t2)


@pytest.mark.parametrize("name,data", list(_cases()))
def test_resumable_matches_one_shot(name, data):
    """Packing driven by receive chunks (PackTap) gives the one-shot stream and table."""
    rng = np.random.default_rng(len(data))
    cuts = sorted(rng.integers(0, len(data) + 1, 7).tolist()) if data else []
    cuts += [64 * 32 * 2, 64 * 33, 5]  # group and block edges, out of order (no-ops)
    one, tab1 = N.text_pack(data)
    got, tab2 = N.text_pack_chunked(data, cuts)
    assert got == one and np.array_equal(tab1, tab2)


def test_ratio_on_jackson_text():
    doc = _jackson_text(4)
    packed, _ = N.text_pack(doc)
    # everything but the envelope and the block holding it packs 2:1
    assert len(packed) < 0.51 * len(doc)


def test_group_table_layout():
    data = b"0" * 64 + b"x" * 64 + b"1" * (64 * 30) + b"2" * 64 + b"tail"
    packed, tab = N.text_pack(data, True)
    # group 0: block 1 raw, the other 31 packed; group 1: block 0 packed + a raw 4-byte tail
    assert tab[0] == 0 and tab[1] == 0xFFFFFFFF & ~0b10
    assert tab[2] == 31 * 32 + 64 and tab[3] == 1
    assert len(packed) == tab[2] + 32 + 4


@pytest.mark.gpu
@pytest.mark.parametrize("name,data", [c for c in _cases() if c[0] != "empty"])
def test_device_unpack_matches_host(name, data):
    import torch

    packed, tab = N.text_pack(data)
    dev = torch.device("cuda", 0)
    p = torch.frombuffer(bytearray(packed + b"\0" * 16), dtype=torch.uint8).to(dev)
    t = torch.from_numpy(tab.astype(np.int64)).to(torch.int32).to(dev)
    # the expansion must write [0, n) only: guard bytes after the span stay untouched
    out = torch.full((len(data) + 64,), 0xA5, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev)
    N.text_unpack(p.data_ptr(), t.data_ptr(), len(data), out.data_ptr(), s.cuda_stream)
    got = bytes(out.cpu().numpy())
    assert got[:len(data)] == data
    assert got[len(data):] == b"\xa5" * 64


@pytest.mark.gpu
def test_device_unpack_reads_host_mapped_packed_text():
    """The GPU ingest's zero-copy form: the packed stream and its group table stay in host-mapped
    pinned memory (the source's pinned chunk) and the kernel reads them over the link."""
    import torch

    data = _jackson_text(3) + b"\x00tail bytes \xff" + _jackson_text(1)
    packed, tab = N.text_pack(data)
    tb = tab.astype(np.uint32).tobytes()
    buf = N.MappedBuffer(len(packed) + 16 + len(tb))
    v = buf.numpy()
    v[:len(packed)] = np.frombuffer(packed, dtype=np.uint8)
    toff = (len(packed) + 15) & ~15
    v[toff:toff + len(tb)] = np.frombuffer(tb, dtype=np.uint8)
    dev = torch.device("cuda", 0)
    out = torch.full((len(data) + 64,), 0xA5, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev)
    N.text_unpack(buf.ptr, buf.ptr + toff, len(data), out.data_ptr(), s.cuda_stream)
    got = bytes(out.cpu().numpy())
    assert got[:len(data)] == data and got[len(data):] == b"\xa5" * 64
