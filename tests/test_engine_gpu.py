"""GPU serving path: the gfx950 JSON parser kernel against the host decoder, and the full
engine (Kafka -> GPU JSON parse -> hipGraph forward -> Kafka) against the fp32 torch oracle."""

import json
import time

import numpy as np
import pytest
import torch

from gale._native import native
from gale.config import GaleConfig
from gale.engine import Engine
from gale.models import fold_params, get_model, init_params
from gale.models.reference import forward

pytestmark = pytest.mark.gpu

C = native()
K = C.kafka
REC = np.dtype([("off", "<i8"), ("len", "<i4"), ("slot", "<i4"), ("images", "<i4"),
                ("status", "<i4"), ("tile0", "<i4"), ("has_cnt", "<i4"), ("cnt_off", "<i8"),
                ("pad", "<i8")])
assert REC.itemsize == C.JSON_RECORD_BYTES


def stage(arrays):
    """Pack JSON array texts 16-byte aligned (+16 slack) and their JsonRecord table."""
    buf = bytearray()
    recs = np.zeros(len(arrays), dtype=REC)
    slot = tiles = 0
    for i, (txt, images) in enumerate(arrays):
        recs[i] = (len(buf), len(txt), slot, images, 0, tiles, 0, 0, 0)
        tiles += C.json_tile_count(len(buf), len(txt))
        buf += txt + b" " * ((-len(txt)) % 16)
        slot += images
    buf += b" " * 16
    return np.frombuffer(bytes(buf), dtype=np.uint8), recs, slot, tiles


def gpu_parse(arrays, H, Wd, Cc):
    raw, recs, total, tiles = stage(arrays)
    tile_rec = np.zeros(max(tiles, 1), dtype=np.int32)
    for i, r in enumerate(recs):
        n = C.json_tile_count(int(r["off"]), int(r["len"]))
        tile_rec[r["tile0"]:r["tile0"] + n] = i
    d_raw = torch.from_numpy(raw.copy()).cuda()
    d_recs = torch.from_numpy(recs.view(np.uint8).copy()).cuda()
    d_tile_rec = torch.from_numpy(tile_rec).cuda()
    d_tiles = torch.zeros(max(tiles, 1), dtype=torch.int32, device="cuda")
    out = torch.full((max(total, 1), H, Wd, Cc), -7.0, device="cuda")
    C.json_parse_instances(len(arrays), tiles, d_recs.data_ptr(), d_tile_rec.data_ptr(),
                           d_raw.data_ptr(), H, Wd, Cc, d_tiles.data_ptr(), out.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    st = d_recs.cpu().numpy().view(REC)["status"]
    return out.cpu().numpy(), st


def array_text(record: bytes, H, Wd, Cc):
    s, off, ln, n = C.scan_instances(record, H, Wd, Cc)
    assert s == 0
    return record[off:off + ln], n


def test_gpu_json_parse_matches_host():
    rng = np.random.default_rng(0)
    H, Wd, Cc = 5, 4, 3
    recs, xs = [], []
    for n in (1, 3, 2):
        x = (rng.standard_normal((n, H, Wd, Cc)) * 10.0 ** rng.integers(-8, 8, (n, H, Wd, Cc))
             ).astype(np.float32)
        xs.append(x)
        recs.append(array_text(C.encode_instances(x), H, Wd, Cc))
    # python's json.dumps formatting (doubles, spaces) must parse too
    x4 = rng.random((2, H, Wd, Cc)).astype(np.float32)
    xs.append(x4)
    recs.append(array_text(json.dumps({"instances": x4.astype(np.float64).tolist()},
                                      indent=1).encode(), H, Wd, Cc))
    out, st = gpu_parse(recs, H, Wd, Cc)
    assert list(st) == [0, 0, 0, 0]
    ref = np.concatenate(xs)
    np.testing.assert_array_equal(out, ref)  # correctly rounded: bit-exact round trip


def test_gpu_json_parse_multi_tile():
    """CIFAR-sized records span many 4 KiB tiles: token indices carry across tiles, tokens
    straddle tile edges, and a whitespace run longer than the LDS halo falls back to global."""
    rng = np.random.default_rng(1)
    H, Wd, Cc = 32, 32, 3
    recs, xs = [], []
    for n in (1, 2, 1):
        x = (rng.standard_normal((n, H, Wd, Cc)) * 10.0 ** rng.integers(-6, 6, (n, H, Wd, Cc))
             ).astype(np.float32)
        xs.append(x)
        recs.append(array_text(C.encode_instances(x), H, Wd, Cc))
    x = rng.random((1, H, Wd, Cc)).astype(np.float32)
    xs.append(x)
    recs.append(array_text(json.dumps({"instances": x.astype(np.float64).tolist()},
                                      indent=2).encode(), H, Wd, Cc))
    x = rng.random((1, H, Wd, Cc)).astype(np.float32)
    xs.append(x)
    txt, n = array_text(C.encode_instances(x), H, Wd, Cc)
    cut = txt.index(b",", 9000)
    recs.append((txt[:cut] + b" " * 300 + txt[cut:cut + 1] + b"\n" * 200 + txt[cut + 1:], n))
    out, st = gpu_parse(recs, H, Wd, Cc)
    assert list(st) == [0] * len(recs)
    np.testing.assert_array_equal(out, np.concatenate(xs))


def test_gpu_json_parse_multi_tile_errors():
    rng = np.random.default_rng(2)
    H, Wd, Cc = 32, 32, 3
    good, n = array_text(C.encode_instances(rng.random((1, H, Wd, Cc)).astype(np.float32)),
                         H, Wd, Cc)
    d = next(i for i in range(20000, len(good)) if good[i:i + 1].isdigit())
    bad_char = good[:d] + b"x" + good[d + 1:]
    k = good.index(b"],[", 30000)
    ragged = good[:k] + b"," + good[k + 3:]                  # two pixels fused: wrong structure
    short = good[:good.rindex(b",")] + b"]]]]"               # last number dropped
    _, st = gpu_parse([(good, n), (bad_char, n), (ragged, n), (short, n), (good, n)], H, Wd, Cc)
    assert list(st) == [0, 2, 3, 1, 0]


@pytest.mark.parametrize("txt,status", [
    (b"[[[[1,2,3],[4,5,6]],[[1,2,3],[4,5,6]]]]", 0),
    (b"[[[[1,2,3],[4,5,6]],[[1,2,3],[4,5]]]]", 1),        # one number short
    (b"[[[[1,2,3],[4,5,6]],[[1,2,3,4],[5,6]]]]", 3),      # ragged: counts match, structure not
    (b"[[[[1,2,3],[4,5,6],[1,2,3],[4,5,6]]]]", 3),        # 1x4 instead of 2x2
    (b"[[[[1,2,3],[4,5,x6]],[[1,2,3],[4,5,6]]]]", 2),     # bad element
    (b"[[[[1,2,3],[4,5,06]],[[1,2,3],[4,5,6]]]]", 2),     # leading zero
    (b"[[[[1,2,3],[4,5,6]],[[1,2,3],[4,5,6]]]],[]", 3),   # trailing junk
])
def test_gpu_json_parse_validates_structure(txt, status):
    _, st = gpu_parse([(txt, 1)], 2, 2, 3)
    assert st[0] == status


@pytest.fixture()
def broker():
    b = K.Broker()
    b.start()
    b.create_topic("in", 1)
    b.create_topic("out", 1)
    yield b
    b.stop()


def run_engine(broker, n, **kw):
    cfg = GaleConfig(topology_name="g", input_topic="in", output_topic="out",
                     bootstrap=f"127.0.0.1:{broker.port}", start_offset="earliest",
                     max_batch=32, max_wait_us=500, **kw)
    eng = Engine(cfg, devices=[0], max_records=n)
    eng.start()
    assert eng.wait(120), eng.stats()
    eng.stop()
    return eng, broker.read("out", 0)


def centered_log(p):
    """Logits up to their per-row constant, recovered from softmax rows."""
    lp = np.log(np.maximum(np.asarray(p, dtype=np.float64), 1e-38))
    return lp - lp.mean(axis=-1, keepdims=True)


@pytest.mark.parametrize("model,ingest", [("resnet20", True), ("resnet20", False),
                                          ("lenet5", True), ("resnet20", "pack"),
                                          ("resnet20", "pack-inplace"), ("lenet5", "pack"),
                                          ("resnet20", "pack-noparse"),
                                          ("resnet20", "pack-plan-dma")])
def test_gpu_engine_matches_oracle(broker, model, ingest, monkeypatch):
    """Every output record is matched to ITS input by key (output_key=input) and compared on
    logits (centered log-softmax) with a bf16-level relative tolerance: a misrouted batch split
    (image i's row under record j) or a wrong image count cannot pass. ingest=True: CRC32C and
    image counts on the GPU and the parser reading the device-resident fetch buffer; False: the
    host decode path with per-batch H2D staging; "pack": GPU ingest of nibble-packed fetch
    bodies (the source's PackTap, expanded on the device before the CRC / count / parse).
    With GPU ingest the records are parsed into the fetch's image arena by the ingest pass and
    the batch step runs the forward alone ("pack-noparse": the step parses, as in round 5).
    "pack-plan-dma": the ingest plan takes its own DMA instead of riding the text's (the path a
    fetch takes when the plan does not fit behind it in its chunk)."""
    pack = ingest in ("pack", "pack-inplace", "pack-noparse", "pack-plan-dma")
    if ingest == "pack-plan-dma":
        monkeypatch.setenv("GALE_INGEST_PLAN_SEPARATE", "1")
    if pack and not C.text_pack_fast():
        pytest.skip("no AVX-512 VBMI on this host")
    net = get_model(model)
    params = init_params(net, seed=0, calib_batch=16)
    rng = np.random.default_rng(1)
    counts = [1, 2, 1, 3, 1, 1, 4, 1, 2, 1] * 3
    xs = {}
    for i, n in enumerate(counts):
        x = rng.random((n,) + net.input_shape, dtype=np.float32)
        xs[f"r{i}".encode()] = x
        broker.append("in", 0, [C.encode_instances(x)], [f"r{i}".encode()])
    broker.append("in", 0, [b'{"instances": [[[[0.5]]]]}'], [b"bad"])  # wrong shape -> null
    cfg = GaleConfig(topology_name="g", input_topic="in", output_topic="out", model=model,
                     bootstrap=f"127.0.0.1:{broker.port}", start_offset="earliest",
                     max_batch=32, max_wait_us=500, output_key="input",
                     gpu_ingest=bool(ingest), text_pack=pack,
                     text_pack_bounce=ingest != "pack-inplace",
                     ingest_parse=ingest != "pack-noparse")
    eng = Engine(cfg, devices=[0], max_records=len(counts) + 1, params=params)
    eng.start()
    assert eng.wait(120), eng.stats()
    eng.stop()
    out = broker.read("out", 0)
    assert len(out) == len(counts) + 1
    by_key = {r["key"]: r["value"] for r in out}
    assert set(by_key) == set(xs) | {b"bad"} and by_key[b"bad"] is None
    folded = fold_params(net, params)
    worst = 0.0
    for k, x in xs.items():
        ref = centered_log(forward(net, folded, torch.from_numpy(x)).numpy())
        got = centered_log(json.loads(by_key[k])["predictions"])
        assert got.shape == ref.shape, k
        rel = np.abs(got - ref).max() / max(np.abs(ref).max(), 1.0)
        worst = max(worst, rel)
        assert np.array_equal(got.argmax(-1), ref.argmax(-1)) or rel < 1e-2, k
    assert worst < 2e-2, worst
    st = eng.stats()
    assert st["errors"] == 1 and st["images_out"] == sum(counts)
    assert (st["ingested_records"] > 0) == bool(ingest)
    # the ingest plan rides the text's DMA (written behind the fetch in its pinned chunk)
    assert (st["ingest_plan_in_chunk"] > 0) == (bool(ingest) and ingest != "pack-plan-dma"), st
    # every good record's images came parsed from the ingest arena (the step ran the forward
    # alone), unless the ingest parse is off or there is no GPU ingest
    want = len(counts) if ingest and ingest != "pack-noparse" else 0
    assert st["ingest_parsed_records"] == want and st["preparsed_records"] == want, st
    # such batches are one forward launch, their inputs in the kernel arguments
    assert (st["table_batches"] > 0) == (want > 0), st
    if pack:  # the text crossed the link packed (~0.5 bytes per fetched byte)
        assert 0 < st["ingest_link_bytes"] < 0.6 * st["ingest_text_bytes"], st
        # the bounce receive left sparse host copies (nothing needed the text on the host)
        assert (st["sparse_fetches"] > 0) == (ingest != "pack-inplace"), st
        assert st["restored_fetches"] == 0, st


@pytest.mark.parametrize("ingest_parse", [True, False])
def test_gpu_ingest_parse_verdicts(broker, ingest_parse):
    """Records the ingest pass parses are judged there: a ragged array whose element count is
    right (one pixel with 2 values, the next with 4) is bad_shape, a malformed number is
    bad_number, a wrong element count is bad_shape - the same verdicts as the step's parse
    (ingest_parse=False), and the good records' predictions are identical either way."""
    rng = np.random.default_rng(3)
    good = {f"g{i}".encode(): rng.random((1 + i % 2, 32, 32, 3), dtype=np.float32)
            for i in range(6)}
    for k, x in good.items():
        broker.append("in", 0, [C.encode_instances(x)], [k])
    x = rng.random((1, 32, 32, 3), dtype=np.float32).tolist()
    x[0][0][1] = x[0][0][1] + [x[0][0][0].pop()]  # pixel (0, 0): 2 values, pixel (0, 1): 4
    ragged = json.dumps({"instances": x}).encode()
    badnum = C.encode_instances(rng.random((1, 32, 32, 3), dtype=np.float32))
    i = badnum.index(b",", 2000)
    badnum = badnum[:i] + b".5.5" + badnum[i:]  # "0.123.5.5": a number with two points
    short = C.encode_instances(rng.random((1, 32, 32, 3), dtype=np.float32))
    short = short[:short.rindex(b",")] + b"]]]]}"  # 3071 elements
    broker.append("in", 0, [ragged, badnum, short], [b"ragged", b"badnum", b"short"])
    n = len(good) + 3
    eng, out = run_engine(broker, n, output_key="input", on_error="error-json",
                          ingest_parse=ingest_parse)
    by_key = {r["key"]: r["value"] for r in out}
    assert len(out) == n
    assert json.loads(by_key[b"ragged"])["error"] == "bad_shape"
    # (a malformed number: its own token fails as a number, and the parser's structural check of
    # the elements around it may speak first - either verdict rejects the record)
    assert json.loads(by_key[b"badnum"])["error"] in ("bad_number", "bad_shape")
    assert json.loads(by_key[b"short"])["error"] == "bad_shape"
    for k, x in good.items():
        p = np.array(json.loads(by_key[k])["predictions"])
        assert p.shape == (len(x), 10) and np.allclose(p.sum(-1), 1.0, atol=1e-4)
    st = eng.stats()
    assert st["errors"] == 3
    assert st["preparsed_records"] == (len(good) if ingest_parse else 0), st
    # identical outputs - predictions and verdicts - with and without the ingest parse (same
    # kernels, same rounding)
    key = "_ingest_parse_preds"
    prev = getattr(test_gpu_ingest_parse_verdicts, key, None)
    cur = dict(by_key)
    if prev is None:
        setattr(test_gpu_ingest_parse_verdicts, key, cur)
    else:
        assert prev == cur


def test_gpu_engine_float_format_java8(broker):
    """--float-format java8 with GPU replicas: the device formatter (JDK 19 rule) is bypassed and
    the engine prints Java 8 Float.toString digits from the fp32 softmax rows."""
    rng = np.random.default_rng(5)
    n = 12
    for i in range(n):
        broker.append("in", 0, [C.encode_instances(rng.random((2, 32, 32, 3), dtype=np.float32))])
    eng, out = run_engine(broker, n, float_format="java8")
    assert len(out) == n and eng.stats()["errors"] == 0
    for r in out:
        p = np.array(json.loads(r["value"])["predictions"], dtype=np.float32)
        assert p.shape == (2, 10)
        assert C.encode_predictions(p, False, True) == r["value"]


def test_gpu_crc32c_chunks_kernel():
    """The ingest CRC kernel: raw CRCs of arbitrary (misaligned, partial) windows, joined into
    standard CRC32Cs, equal the host's."""
    import os

    buf = os.urandom(3 * 4096 + 777)
    d = torch.frombuffer(bytearray(buf + bytes(64)), dtype=torch.uint8).cuda()
    tables = torch.tensor(np.array(K.crc32c_device_tables(), dtype=np.uint32).view(np.int32),
                          device="cuda")
    regions = [(0, 1), (5, 4096), (21, 9000), (3, len(buf) - 3)]
    wins, plan = [], []
    for s0, ln in regions:
        n = -(-ln // 4096)
        plan.append((s0, ln, len(wins), n))
        for k in range(n):
            wins.append((s0 + ln - 4096 * (n - 1 - k), ln - 4096 * (n - 1) if k == 0 else 4096))
    ch = np.zeros(len(wins), dtype=[("end", "<i8"), ("len", "<i4"), ("pad", "<i4")])
    for i, (e, ln) in enumerate(wins):
        ch[i] = (e, ln, 0)
    dch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
    out = torch.zeros(len(wins), dtype=torch.int32, device="cuda")
    C.crc32c_chunks(d.data_ptr(), dch.data_ptr(), len(wins), tables.data_ptr(), out.data_ptr(),
                    torch.cuda.current_stream().cuda_stream)
    raw_w = out.cpu().numpy().view(np.uint32)
    for s0, ln, first, n in plan:
        raw = 0
        for k in range(n):
            c = int(raw_w[first + k])
            raw = c if k == 0 else K.crc32c_shift(raw, 4096) ^ c
        std = raw ^ K.crc32c_shift(0xFFFFFFFF, ln) ^ 0xFFFFFFFF
        assert std == K.crc32c(buf[s0:s0 + ln]), (s0, ln)


def host_tile_tokens(buf, off, ln):
    """Number tokens starting in each 2 KiB tile of the record text at [off, off + ln) (tiles
    counted from the 16-byte-aligned start, as json_tile_count)."""
    abeg = off & ~15
    b = np.frombuffer(buf, dtype=np.uint8)[abeg:off + ln].copy()
    beg = off - abeg
    delim = np.isin(b, np.frombuffer(b"[], \t\r\n", dtype=np.uint8))
    delim[:beg] = True
    prev = np.concatenate([[True], delim[:-1]])
    start = ~delim & prev
    nt = C.json_tile_count(off, ln)
    T = C.JSON_TILE_BYTES
    return np.array([start[k * T:(k + 1) * T].sum() for k in range(nt)], dtype=np.int64)


def test_gpu_fused_ingest_kernel_matches_separate_passes():
    """ingest_crc_count (CRC windows + token counts in ONE launch, one workgroup per group of
    GROUP_TILES tiles) produces the raw window CRCs of crc32c_chunks, every record's count block
    (tile token counts as counted on the host, then one sum per tile group) and the group sums
    the host adds per record; the parse then reuses those blocks (has_cnt, no counting launch)
    and decodes the same tensor. Records of 1-3 CIFAR images and one ImageNet image (~850
    tiles)."""
    import os

    rng = np.random.default_rng(8)
    G = C.GROUP_TILES
    cases = [(32, 32, 3, (1, 3, 2)), (224, 224, 3, (1,))]
    for H, Wd, Cc, ns in cases:
        xs = [rng.random((n, H, Wd, Cc), dtype=np.float32) for n in ns]
        arrays = [array_text(C.encode_instances(x), H, Wd, Cc) for x in xs]
        raw, recs, total, tiles = stage(arrays)
        buf = bytes(raw) + os.urandom(5000)
        wins = [(len(buf) - 4096 * k, 4096) for k in range(len(buf) // 4096)][::-1]
        wins = [(len(buf) - 4096 * len(wins), len(buf) % 4096)] + wins if len(buf) % 4096 else wins
        ch = np.zeros(len(wins), dtype=[("end", "<i8"), ("len", "<i4"), ("pad", "<i4")])
        for i, (e, ln) in enumerate(wins):
            ch[i] = (e, ln, 0)
        groups, grp0 = [], []
        for i, r in enumerate(recs):
            grp0.append(len(groups))
            nt = C.json_tile_count(int(r["off"]), int(r["len"]))
            groups += [(i, t0) for t0 in range(0, nt, G)]
        recs["pad"] = grp0  # JsonRecord::grp0
        d = torch.frombuffer(bytearray(buf + bytes(64)), dtype=torch.uint8).cuda()
        tables = torch.tensor(np.array(K.crc32c_device_tables(), dtype=np.uint32).view(np.int32),
                              device="cuda")
        dch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
        dgrp = torch.tensor(np.array(groups, dtype=np.int32).reshape(-1), device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        drec = torch.from_numpy(recs.view(np.uint8).copy()).cuda()
        crc = torch.zeros(len(wins), dtype=torch.int32, device="cuda")
        cnt = torch.full((tiles + len(groups),), -1, dtype=torch.int32, device="cuda")
        gsum = torch.full((len(groups),), -1, dtype=torch.int32, device="cuda")
        C.ingest_crc_count(d.data_ptr(), dch.data_ptr(), len(wins), tables.data_ptr(),
                           crc.data_ptr(), len(recs), len(groups), drec.data_ptr(),
                           dgrp.data_ptr(), cnt.data_ptr(), gsum.data_ptr(), s)
        crc2 = torch.zeros(len(wins), dtype=torch.int32, device="cuda")
        C.crc32c_chunks(d.data_ptr(), dch.data_ptr(), len(wins), tables.data_ptr(),
                        crc2.data_ptr(), s)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(crc.cpu().numpy(), crc2.cpu().numpy())
        gs = gsum.cpu().numpy()
        bounds = grp0 + [len(groups)]
        assert [gs[bounds[i]:bounds[i + 1]].sum() for i in range(len(recs))] == \
            [len(x) * H * Wd * Cc for x in xs]
        assert list(drec.cpu().numpy().view(REC)["status"]) == [0] * len(recs)
        c = cnt.cpu().numpy()
        for i, r in enumerate(recs):
            want = host_tile_tokens(buf, int(r["off"]), int(r["len"]))
            nt = len(want)
            blk = c[int(r["tile0"]) + grp0[i]:]
            np.testing.assert_array_equal(blk[:nt], want)
            sums = [want[t0:t0 + G].sum() for t0 in range(0, nt, G)]
            np.testing.assert_array_equal(blk[nt:nt + len(sums)], sums)
            np.testing.assert_array_equal(gs[bounds[i]:bounds[i + 1]], sums)
        # parse with the ingest blocks (has_cnt, cnt_off = block start), no count pass
        recs2 = recs.copy()
        recs2["has_cnt"] = 1
        recs2["cnt_off"] = [cnt.data_ptr() + 4 * (int(r["tile0"]) + grp0[i]) - d.data_ptr()
                            for i, r in enumerate(recs)]
        drec = torch.from_numpy(recs2.view(np.uint8).copy()).cuda()
        tile_rec = np.zeros(tiles, dtype=np.int32)
        for i, r in enumerate(recs):
            n = C.json_tile_count(int(r["off"]), int(r["len"]))
            tile_rec[r["tile0"]:r["tile0"] + n] = i
        dmap = torch.from_numpy(tile_rec).cuda()
        out = torch.full((total, H, Wd, Cc), -7.0, device="cuda")
        scratch = torch.full((tiles,), 123456, dtype=torch.int32, device="cuda")  # unused
        C.json_parse_instances(len(recs), tiles, drec.data_ptr(), dmap.data_ptr(), d.data_ptr(),
                               H, Wd, Cc, scratch.data_ptr(), out.data_ptr(), s,
                               count_pass=False)
        torch.cuda.synchronize()
        assert list(drec.cpu().numpy().view(REC)["status"]) == [0] * len(recs)
        np.testing.assert_array_equal(out.cpu().numpy(), np.concatenate(xs))


@pytest.mark.parametrize("tail", [5000, 4097, 61])
def test_gpu_fused_packed_ingest_matches_plain(tail):
    """ingest_crc_count over a nibble-packed body (text_unpack folded in): the window CRCs
    equal crc32c_chunks over the plain text, the count blocks and group sums equal the plain
    pass's, and every record's 16-byte-aligned extent is stored into the text image (what the
    parse reads) byte for byte. Random bytes after the records make raw blocks, and the body
    length leaves a raw partial final block."""
    import os

    rng = np.random.default_rng(12)
    G = C.GROUP_TILES
    H, Wd, Cc = 32, 32, 3
    xs = [rng.random((n, H, Wd, Cc), dtype=np.float32) for n in (1, 3, 2, 1)]
    arrays = [array_text(C.encode_instances(x), H, Wd, Cc) for x in xs]
    raw, recs, total, tiles = stage(arrays)
    buf = os.urandom(48) + bytes(raw) + os.urandom(tail)
    recs["off"] += 48
    recs["tile0"] = np.cumsum([0] + [C.json_tile_count(int(r["off"]), int(r["len"]))
                                     for r in recs][:-1])
    tiles = sum(C.json_tile_count(int(r["off"]), int(r["len"])) for r in recs)
    wins = [(len(buf) - 4096 * k, 4096) for k in range(len(buf) // 4096)][::-1]
    if len(buf) % 4096:
        wins = [(len(buf) - 4096 * len(wins), len(buf) % 4096)] + wins
    wins = [(1000, 900), (2000, 5)] + wins  # unaligned short windows too
    groups, grp0 = [], []
    for i, r in enumerate(recs):
        grp0.append(len(groups))
        nt = C.json_tile_count(int(r["off"]), int(r["len"]))
        groups += [(i, t0) for t0 in range(0, nt, G)]
    recs["pad"] = grp0
    ch = np.zeros(len(wins), dtype=[("end", "<i8"), ("len", "<i4"), ("pad", "<i4")])
    for i, (e, ln) in enumerate(wins):
        ch[i] = (e, ln, 0)
    packed, tab = C.text_pack(buf)
    s = torch.cuda.current_stream().cuda_stream
    tables = torch.tensor(np.array(K.crc32c_device_tables(), dtype=np.uint32).view(np.int32),
                          device="cuda")
    dch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
    dgrp = torch.tensor(np.array(groups, dtype=np.int32).reshape(-1), device="cuda")
    dp = torch.frombuffer(bytearray(packed + bytes(64)), dtype=torch.uint8).cuda()
    dt = torch.from_numpy(tab.astype(np.int64)).to(torch.int32).cuda()
    out = torch.full((len(buf) + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    results = {}
    for mode in ("plain", "packed"):
        d = torch.frombuffer(bytearray(buf + bytes(64)), dtype=torch.uint8).cuda()
        drec = torch.from_numpy(recs.view(np.uint8).copy()).cuda()
        crc = torch.zeros(len(wins), dtype=torch.int32, device="cuda")
        cnt = torch.full((tiles + len(groups),), -1, dtype=torch.int32, device="cuda")
        gsum = torch.full((len(groups),), -1, dtype=torch.int32, device="cuda")
        gbad = torch.full((len(groups),), -1, dtype=torch.int32, device="cuda")
        kw = dict(gbad=gbad.data_ptr())
        if mode == "packed":
            kw.update(packed=dp.data_ptr(), tab=dt.data_ptr(), text_out=out.data_ptr())
        C.ingest_crc_count(d.data_ptr(), dch.data_ptr(), len(wins), tables.data_ptr(),
                           crc.data_ptr(), len(recs), len(groups), drec.data_ptr(),
                           dgrp.data_ptr(), cnt.data_ptr(), gsum.data_ptr(), s, **kw)
        torch.cuda.synchronize()
        results[mode] = [t.cpu().numpy() for t in (crc, cnt, gsum, gbad)]
    for a, b in zip(results["plain"], results["packed"]):
        np.testing.assert_array_equal(a, b)
    assert (results["packed"][3] == 0).all()
    raw_w = results["packed"][0].view(np.uint32)
    for i, (e, ln) in enumerate(wins):  # (the plain pass's CRCs are right: checked elsewhere)
        std = int(raw_w[i]) ^ K.crc32c_shift(0xFFFFFFFF, ln) ^ 0xFFFFFFFF
        assert std == K.crc32c(buf[e - ln:e]), (e, ln)
    got = out.cpu().numpy()
    src = np.frombuffer(buf, dtype=np.uint8)
    for r in recs:
        a0 = int(r["off"]) & ~15
        a1 = (int(r["off"]) + int(r["len"]) + 15) & ~15
        np.testing.assert_array_equal(got[a0:a1], src[a0:a1])


def test_gpu_ingest_zero_copy_plan_and_group_verdicts():
    """The engine's zero-copy form of ingest_crc_count: windows, records and groups are read from
    host-mapped pinned memory, CRCs / group sums / group verdicts are stored back into it (no
    copies, no atomics on host memory). A record with a byte outside the number alphabet gets
    verdict 2 on exactly the group holding that byte; the others stay 0 and their sums match."""
    import os

    rng = np.random.default_rng(11)
    G = C.GROUP_TILES
    H, Wd, Cc = 32, 32, 3
    xs = [rng.random((n, H, Wd, Cc), dtype=np.float32) for n in (2, 1, 3)]
    arrays = [array_text(C.encode_instances(x), H, Wd, Cc) for x in xs]
    raw, recs, total, tiles = stage(arrays)
    raw = bytearray(raw)
    bad_pos = int(recs[1]["off"]) + 9000  # inside record 1, tile 4 (group 1)
    while raw[bad_pos] not in b"0123456789":
        bad_pos += 1
    raw[bad_pos] = ord("x")
    buf = bytes(raw) + os.urandom(3000)
    wins = [(len(buf) - 4096 * k, 4096) for k in range(len(buf) // 4096)][::-1]
    if len(buf) % 4096:
        wins = [(len(buf) - 4096 * len(wins), len(buf) % 4096)] + wins
    groups, grp0 = [], []
    for i, r in enumerate(recs):
        grp0.append(len(groups))
        nt = C.json_tile_count(int(r["off"]), int(r["len"]))
        groups += [(i, t0) for t0 in range(0, nt, G)]
    recs["pad"] = grp0
    ch = np.zeros(len(wins), dtype=[("end", "<i8"), ("len", "<i4"), ("pad", "<i4")])
    for i, (e, ln) in enumerate(wins):
        ch[i] = (e, ln, 0)
    # plan and results in ONE host-mapped buffer, as GpuIngest lays them out
    parts = [np.frombuffer(a.tobytes(), dtype=np.uint8)
             for a in (ch, np.array(groups, dtype=np.int32), recs)]
    offs, o = [], 0
    for a in parts:
        offs.append(o)
        o += (a.nbytes + 15) & ~15
    o_gsum = o
    o_crc = o_gsum + ((4 * len(groups) + 15) & ~15)
    o_gbad = o_crc + ((4 * len(wins) + 15) & ~15)
    mb = C.MappedBuffer(o_gbad + 4 * len(groups) + 16)
    v = mb.numpy()
    for a, off in zip(parts, offs):
        v[off:off + a.nbytes] = a
    v[o_gsum:] = 0xEE  # (results must overwrite this)
    d = torch.frombuffer(bytearray(buf + bytes(64)), dtype=torch.uint8).cuda()
    tables = torch.tensor(np.array(K.crc32c_device_tables(), dtype=np.uint32).view(np.int32),
                          device="cuda")
    cnt = torch.full((tiles + len(groups),), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    C.ingest_crc_count(d.data_ptr(), mb.ptr + offs[0], len(wins), tables.data_ptr(),
                       mb.ptr + o_crc, len(recs), len(groups), mb.ptr + offs[2],
                       mb.ptr + offs[1], cnt.data_ptr(), mb.ptr + o_gsum, s,
                       gbad=mb.ptr + o_gbad)
    torch.cuda.synchronize()
    gbad = v[o_gbad:o_gbad + 4 * len(groups)].view(np.int32)
    gsum = v[o_gsum:o_gsum + 4 * len(groups)].view(np.int32)
    want_bad = [2 if (i == 1 and t0 == 4) else 0 for i, t0 in groups]
    assert list(gbad) == want_bad
    assert list(v[offs[2]:offs[2] + recs.nbytes].view(REC)["status"]) == [0, 0, 0]  # untouched
    for i, r in enumerate(recs):
        if i == 1:
            continue
        g0, g1 = grp0[i], (grp0[i + 1] if i + 1 < len(recs) else len(groups))
        assert gsum[g0:g1].sum() == len(xs[i]) * H * Wd * Cc
    crc = v[o_crc:o_crc + 4 * len(wins)].view(np.int32)
    crc2 = torch.zeros(len(wins), dtype=torch.int32, device="cuda")
    dch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
    C.crc32c_chunks(d.data_ptr(), dch.data_ptr(), len(wins), tables.data_ptr(), crc2.data_ptr(),
                    s)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(crc, crc2.cpu().numpy())


def test_gpu_ingest_rejects_corrupt_batch_and_counts_images(broker):
    """GPU ingest: a bit flip inside a record batch fails its device-computed CRC32C, so all of
    its records get the error policy; records of intact batches are counted (N = 2 images
    each, from the GPU token count) and served from the device-resident fetch buffer."""
    rng = np.random.default_rng(5)
    recs = [C.encode_instances(rng.random((2, 32, 32, 3), dtype=np.float32)) for _ in range(6)]
    good = K.encode_batch([(None, r, -1, None) for r in recs[:3]], 0, 0)
    bad = bytearray(K.encode_batch([(None, r, -1, None) for r in recs[3:]], 0, 0))
    bad[len(bad) // 2] ^= 0x01
    broker.append_batch_repeated("in", 0, good, 1)
    broker.append_batch_repeated("in", 0, bytes(bad), 1)
    eng, out = run_engine(broker, 6, on_error="error-json")
    vals = [r["value"] for r in out]
    assert sum(b"predictions" in v for v in vals) == 3
    assert [json.loads(v)["error"] for v in vals if b"predictions" not in v] == \
        ["corrupt"] * 3
    st = eng.stats()
    assert st["ingested_records"] == 6 and st["images_out"] == 6


def test_gpu_engine_two_replicas_on_one_gpu_and_crash(broker):
    x = np.random.default_rng(2).random((1, 32, 32, 3), dtype=np.float32)
    rec = C.encode_instances(x)
    for _ in range(300):
        broker.append("in", 0, [rec])
    cfg = GaleConfig(topology_name="g", input_topic="in", output_topic="out",
                     bootstrap=f"127.0.0.1:{broker.port}", start_offset="earliest",
                     max_batch=32, max_wait_us=500, replicas=2, fault="replica_crash@4",
                     max_restarts=1, restart_backoff_ms=20)
    eng = Engine(cfg, devices=[0], max_records=300)
    eng.start()
    assert eng.wait(120), eng.stats()
    deadline = time.time() + 10  # the record target can be met before the backoff ends
    while eng.stats()["replica_restarts"] < 1 and time.time() < deadline:
        time.sleep(0.01)
    eng.stop()
    out = broker.read("out", 0)
    assert len(out) == 300 and all(r["value"] is not None for r in out)
    st = eng.stats()
    # the crashed GPU replica was recovered by the supervisor (streams drained) and rejoined
    assert st["replica_failures"] == 1 and st["replica_restarts"] == 1
    assert st["replicas_alive"] == 2
    vals = {r["value"] for r in out}
    assert len(vals) == 1  # identical input -> identical output on both replicas


def test_gpu_locality_split_steals_parse_from_host_pinned():
    """Single-process multi-GPU dispatch on one device (--locality-split 2): two locality slots,
    each with its own source, batcher and pinned fetch pool mirrored on the GPU. All input is in
    partition 0 (slot 0's source), so slot 1's replica is idle and steals from slot 0's queue
    (Storm's load-aware shuffle over every replica, MainTopology.java:62). A stolen record is
    not resident in slot 1's mirror: its text is DMA'd from the host-pinned fetch buffer, as
    across GPUs. Every record is answered exactly once and matches the fp32 oracle by key."""
    net = get_model("resnet20")
    params = init_params(net, seed=0, calib_batch=16)
    b = K.Broker()
    b.start()
    try:
        b.create_topic("in", 2)
        b.create_topic("out", 1)
        rng = np.random.default_rng(7)
        distinct = rng.random((48,) + net.input_shape, dtype=np.float32)
        enc = [C.encode_instances(distinct[i:i + 1]) for i in range(len(distinct))]
        n = 3000  # (a deep backlog in slot 0's partition: slot 1 steals whenever it idles)
        for s in range(0, n, 50):
            b.append("in", 0, [enc[i % len(enc)] for i in range(s, s + 50)],
                     [f"k{i}".encode() for i in range(s, s + 50)])
        cfg = GaleConfig(topology_name="g", input_topic="in", output_topic="out",
                         bootstrap=f"127.0.0.1:{b.port}", start_offset="earliest",
                         max_batch=32, max_wait_us=300, output_key="input", replicas=2,
                         source_parallelism=2, locality_split=2, decode_threads=2,
                         text_pack=False)  # (a stolen record is parsed from its host text)
        eng = Engine(cfg, devices=[0], max_records=n, params=params)
        eng.start()
        assert eng.wait(180), eng.stats()
        eng.stop()
        st = eng.stats()
        reps = eng.replica_stats()
        out = b.read("out", 0)
    finally:
        b.stop()
    assert st["locality_slots"] == 2 and st["steals"] > 0, st
    by_slot = {r["slot"]: r for r in reps}
    assert by_slot[1]["records"] > 0 and by_slot[1]["host_records"] == by_slot[1]["records"]
    assert by_slot[0]["resident_records"] > 0
    keys = [r["key"] for r in out]
    assert len(keys) == n and len(set(keys)) == n  # no loss, no duplicate
    ref = centered_log(forward(net, fold_params(net, params), torch.from_numpy(distinct)).numpy())
    worst = 0.0
    for r in out:
        i = int(r["key"][1:]) % len(distinct)
        got = centered_log(json.loads(r["value"])["predictions"])[0]
        worst = max(worst, np.abs(got - ref[i]).max() / max(np.abs(ref[i]).max(), 1.0))
    assert worst < 2e-2, worst


@pytest.mark.parametrize("ingest", [True, False])
def test_gpu_engine_record_over_max_batch(broker, ingest):
    """A 300-image CIFAR record between small ones (max_batch 128): split over consecutive
    micro-batches on the GPU replicas and reassembled into ONE prediction record, every row
    matched to the fp32 oracle in image order; no TOO_LARGE."""
    net = get_model("resnet20")
    params = init_params(net, seed=0, calib_batch=16)
    rng = np.random.default_rng(7)
    xs = {b"a": rng.random((3, 32, 32, 3), dtype=np.float32),
          b"big": rng.random((300, 32, 32, 3), dtype=np.float32),
          b"b": rng.random((1, 32, 32, 3), dtype=np.float32)}
    for k, x in xs.items():
        broker.append("in", 0, [C.encode_instances(x)], [k])
    cfg = GaleConfig(topology_name="g", input_topic="in", output_topic="out",
                     bootstrap=f"127.0.0.1:{broker.port}", start_offset="earliest",
                     max_batch=128, max_wait_us=500, output_key="input", gpu_ingest=ingest)
    eng = Engine(cfg, devices=[0], max_records=3, params=params)
    eng.start()
    assert eng.wait(120), eng.stats()
    eng.stop()
    out = {r["key"]: r["value"] for r in broker.read("out", 0)}
    assert set(out) == set(xs)
    folded = fold_params(net, params)
    for k, x in xs.items():
        ref = centered_log(forward(net, folded, torch.from_numpy(x)).numpy())
        got = centered_log(json.loads(out[k])["predictions"])
        assert got.shape == ref.shape, k
        rel = np.abs(got - ref).max() / max(np.abs(ref).max(), 1.0)
        assert rel < 2e-2, (k, rel)
    st = eng.stats()
    assert st["split_records"] == 1 and st["split_fragments"] == 3
    assert st["errors"] == 0 and st["images_out"] == 304 and st["err_too_large"] == 0


@pytest.mark.parametrize("model", ["resnet20", "lenet5"])
def test_gpu_step_graph_equals_eager(model):
    """The captured per-slot step graph (metadata H2D, parse, forward, format, status D2H in one
    hipGraphLaunch, counts read from the metadata header) produces byte-identical output records
    to the op-by-op launches, over batches of every size and with a malformed record inside."""
    net = get_model(model)
    params = init_params(net, seed=0, calib_batch=16)
    rng = np.random.default_rng(21)
    recs = []
    for i in range(40):
        x = rng.random((1 + i % 5,) + net.input_shape, dtype=np.float32)
        recs.append((f"r{i}".encode(), C.encode_instances(x)))
    recs.insert(17, (b"bad", b'{"instances": [[[[0.5, x]]]]}'))
    outs = {}
    for step in (True, False):
        b = K.Broker()
        b.start()
        b.create_topic("in", 1)
        b.create_topic("out", 1)
        for k, v in recs:
            b.append("in", 0, [v], [k])
        cfg = GaleConfig(topology_name="s", input_topic="in", output_topic="out", model=model,
                         bootstrap=f"127.0.0.1:{b.port}", start_offset="earliest",
                         max_batch=32, max_wait_us=300, output_key="input", graph_step=step,
                         on_error="error-json")
        eng = Engine(cfg, devices=[0], max_records=len(recs), params=params)
        eng.start()
        assert eng.wait(120), eng.stats()
        eng.stop()
        st = eng.stats()
        assert (st["graph_step_batches"] == st["batches"]) if step else \
            st["graph_step_batches"] == 0
        outs[step] = {r["key"]: r["value"] for r in b.read("out", 0)}
        b.stop()
    assert outs[True] == outs[False] and len(outs[True]) == len(recs)
    assert b"error" in outs[True][b"bad"]


def test_gpu_pinned_pool_backpressure(broker):
    """A pinned-fetch budget of two buffers: when both are held by queued records the sources
    wait for one to be released instead of staging fetches through the heap (which would send
    those records down the host path and, under load, keep the pool exhausted - the ResNet-50
    regression of profiles/archive/r4_ab_resnet50_lenet_sink.jsonl). Every record is still served by GPU
    ingest, correctly."""
    if not C.text_pack_fast():
        pytest.skip("no AVX-512 VBMI on this host")
    net = get_model("resnet20")
    params = init_params(net, seed=0, calib_batch=16)
    rng = np.random.default_rng(5)
    xs = {}
    for i in range(120):
        x = rng.random((1 + i % 3,) + net.input_shape, dtype=np.float32)
        xs[f"b{i}".encode()] = x
        broker.append("in", 0, [C.encode_instances(x)], [f"b{i}".encode()])
    # 128 KB fetches: a packed chunk is 2.37 MB, so 3 MB (x2 with the pack) = 2 chunks
    cfg = GaleConfig(topology_name="g", input_topic="in", output_topic="out", model="resnet20",
                     bootstrap=f"127.0.0.1:{broker.port}", start_offset="earliest",
                     max_batch=32, max_wait_us=500, output_key="input", gpu_ingest=True,
                     text_pack=True, fetch_max_kb=128, partition_max_kb=128, pinned_fetch_mb=3)
    eng = Engine(cfg, devices=[0], max_records=len(xs), params=params)
    eng.start()
    assert eng.wait(120), eng.stats()
    eng.stop()
    st = eng.stats()
    out = {r["key"]: r["value"] for r in broker.read("out", 0)}
    assert set(out) == set(xs)
    folded = fold_params(net, params)
    for k in list(xs)[::7]:
        ref = centered_log(forward(net, folded, torch.from_numpy(xs[k])).numpy())
        got = centered_log(json.loads(out[k])["predictions"])
        assert np.abs(got - ref).max() / max(np.abs(ref).max(), 1.0) < 2e-2, k
    assert st["pinned_chunks"] <= 2, st
    assert st["pinned_heap_budget"] == 0 and st["pinned_heap_too_large"] == 0, st
    assert st["ingested_records"] == st["records_in"] == len(xs), st


@pytest.mark.parametrize("pack", [True, False])
def test_gpu_engine_resnet50_imagenet_records(broker, pack):
    """ImageNet-size records (224x224x3, ~1.7 MB of JSON per image, ~850 parse tiles) through the
    whole engine: the bounce receive + device text expansion (pack) or raw fetch bodies, the
    grouped ingest count (a record spans many 4-tile groups; the parse takes each tile's first
    element index from the group sums), the parse and the ResNet-50 forward. Outputs are
    key-matched to the same replica's forward of the original float32 tensors."""
    from gale.parallel.weights import materialize_weights
    from gale.runtime.replica import ModelReplica

    if pack and not C.text_pack_fast():
        pytest.skip("no AVX-512 VBMI on this host")
    net = get_model("resnet50")
    params = init_params(net, seed=3, calib_batch=4)
    rng = np.random.default_rng(4)
    xs = {}
    for i, n in enumerate([1, 2, 1]):
        x = rng.random((n,) + net.input_shape, dtype=np.float32)
        xs[f"i{i}".encode()] = x
        broker.append("in", 0, [C.encode_instances(x)], [f"i{i}".encode()])
    cfg = GaleConfig(topology_name="g", input_topic="in", output_topic="out", model="resnet50",
                     bootstrap=f"127.0.0.1:{broker.port}", start_offset="earliest",
                     max_batch=8, max_wait_us=2000, output_key="input", gpu_ingest=True,
                     text_pack=pack)
    eng = Engine(cfg, devices=[0], max_records=len(xs), params=params)
    eng.start()
    assert eng.wait(180), eng.stats()
    eng.stop()
    st = eng.stats()
    assert st["errors"] == 0 and st["ingested_records"] == len(xs), st
    if pack:
        assert st["sparse_fetches"] > 0 and st["restored_fetches"] == 0, st
    out = {r["key"]: r["value"] for r in broker.read("out", 0)}
    assert set(out) == set(xs)
    rep = ModelReplica(net, materialize_weights(net, torch.device("cuda", 0), params=params),
                       max_batch=8, slots=1)
    for k, x in xs.items():
        want = rep.infer_eager(torch.from_numpy(x)).cpu().numpy()
        got = np.array(json.loads(out[k])["predictions"], dtype=np.float32)
        assert got.shape == want.shape, k
        # same kernels, the same floats in (the GPU parse is exact): equal up to a kernel
        # choice that may differ with the batch size
        np.testing.assert_allclose(got, want, rtol=2e-3, atol=1e-6, err_msg=k.decode())
