"""Host-side model zoo checks: shapes, parameter counts, BN folding, packing, plan liveness."""

import pytest
import torch

from gale.models import MODELS, build_plan, fold_params, get_model, init_params, pack_params
from gale.models.graph import Conv, conv_n_tiles, param_layout, stored_channels
from gale.models.reference import forward


def test_param_counts_and_macs():
    counts = {}
    for name in MODELS:
        net = get_model(name)
        p = init_params(net, calibrate=False)
        counts[name] = sum(v.numel() for k, v in p.items() if ".bn." not in k)
    assert counts["lenet5"] == 61706
    assert 0.26e6 < counts["resnet20"] < 0.28e6
    assert 25.4e6 < counts["resnet50"] < 25.6e6
    assert abs(get_model("resnet20").macs_per_image() - 40.55e6) < 0.1e6
    assert abs(get_model("resnet50").macs_per_image() - 4.09e9) < 0.02e9


def test_bn_folding_is_exact_in_fp32():
    net = get_model("resnet20")
    p = init_params(net, seed=3, calib_batch=8)
    x = torch.rand(4, 32, 32, 3)
    a = forward(net, p, x, folded=False)
    b = forward(net, fold_params(net, p), x, folded=True)
    assert torch.allclose(a, b, atol=1e-5)
    assert torch.allclose(a.sum(1), torch.ones(4), atol=1e-5)


def test_calibrated_network_is_not_degenerate():
    net = get_model("resnet20")
    p = init_params(net, seed=0)
    probs = forward(net, fold_params(net, p), torch.rand(32, 32, 32, 3))
    assert probs.max().item() < 0.9999  # not one-hot saturated
    assert probs.min().item() > 1e-6


def test_packing_layout_and_values():
    net = get_model("lenet5")
    f = fold_params(net, init_params(net))
    buf = pack_params(net, f)
    layout, total = param_layout(net)
    assert buf.numel() == total
    for e in layout.values():
        assert e.offset % 256 == 0
    e = layout["conv2.w"]
    w = buf[e.offset:e.offset + e.nbytes].view(torch.bfloat16).reshape(e.shape).float()
    ref = f["conv2.weight"]  # [16, 6, 5, 5]; packed k = (kh*5+kw)*8 + ci
    for (co, ci, kh, kw) in [(0, 0, 0, 0), (15, 5, 4, 4), (3, 2, 1, 3)]:
        got = w[co, (kh * 5 + kw) * 8 + ci]
        assert abs(got - ref[co, ci, kh, kw].to(torch.bfloat16).float()) < 1e-6
    assert w[0, 6].item() == 0.0  # padded input channel
    assert w[16:].abs().sum().item() == 0.0  # padded output rows


@pytest.mark.parametrize("name", list(MODELS))
def test_plan_liveness_never_aliases(name):
    net = get_model(name)
    ops, buf_bytes = build_plan(net, 0)
    for op in ops:
        ids = [op["in"], op["out"]] + ([op["res"]] if op.get("res", -1) >= 0 else [])
        assert len(set(ids)) == len(ids), op
        if op["kind"] == 0:
            c = op["conv"]
            assert c["Kpad"] % 32 == 0 and c["Cout"] % 4 == 0
            assert c["Npad"] % (16 * conv_n_tiles(c["Cout"])) == 0
    assert ops[-1]["out"] == 1
    # (+1: a fused projection keeps its block input alive until conv3)
    assert len(buf_bytes) <= 7


def test_stored_channels():
    assert stored_channels(6) == 8 and stored_channels(84) == 88 and stored_channels(64) == 64


def test_resnet20_plan_is_one_fused_kernel():
    from gale.models.graph import OP_RESNET20, is_cifar_resnet20

    net = get_model("resnet20")
    assert is_cifar_resnet20(net) and not is_cifar_resnet20(get_model("lenet5"))
    ops, buf_bytes = build_plan(net, 1 << 20)
    assert len(ops) == 1 and ops[0]["kind"] == OP_RESNET20 and len(ops[0]["ptrs"]) == 40
    assert buf_bytes == [32 * 32 * 3 * 4, 40]
    layered, _ = build_plan(net, 1 << 20, fused=False)
    convs = [op for op in layered if op["kind"] == 0]
    assert [op["w"] for op in convs] == ops[0]["ptrs"][:19]
    assert [op["bias"] for op in convs] == ops[0]["ptrs"][19:38]


@pytest.mark.parametrize("name", ["resnet20", "resnet50"])
def test_unfolded_bn_plan_structure(name):
    """fold_bn=False: every BatchNorm conv is followed by one in-place bn_act op that carries
    the BN affine, the residual and the ReLU; the conv itself is linear."""
    from gale.models import unfolded_params
    from gale.models.graph import OP_BN_ACT, OP_CONV

    net = get_model(name)
    params = init_params(net, seed=3, calib_batch=2)
    ops, _ = build_plan(net, 0, fold_bn=False)
    bn_convs = [L for L in net.layers if isinstance(L, Conv) and L.bn]
    bn_ops = [i for i, o in enumerate(ops) if o["kind"] == OP_BN_ACT]
    assert len(bn_ops) == len(bn_convs) > 0
    for i, L in zip(bn_ops, bn_convs):
        conv, bn = ops[i - 1], ops[i]
        assert conv["kind"] == OP_CONV and conv["conv"]["relu"] == 0 and conv["res"] == -1
        assert "has_res" not in conv["conv"]
        assert bn["in"] == bn["out"] == conv["out"] and bn["p"][3] == int(L.relu)
        assert (bn["res"] >= 0) == (L.residual is not None) and bn["res"] != bn["out"]
    layout, total = param_layout(net, "bf16", fold_bn=False)
    u = unfolded_params(net, params)
    buf = pack_params(net, u, "bf16", fold_bn=False)
    assert buf.numel() == total
    L = bn_convs[-1]
    e = layout[f"{L.name}.bn_s"]
    got = buf[e.offset: e.offset + e.nbytes].view(torch.float32)[: L.cout]
    assert torch.equal(got, u[f"{L.name}.bn_scale"])
    # the affine after the raw conv is the folded conv, exactly in fp32 algebra
    f = fold_params(net, params)
    s, t = u[f"{L.name}.bn_scale"], u[f"{L.name}.bn_shift"]
    assert torch.allclose(u[f"{L.name}.bias"] * s + t, f[f"{L.name}.bias"], atol=1e-5)
    with pytest.raises(ValueError):
        param_layout(net, "fp8", fold_bn=False)
    # fp32 unfolded plan: fp32 weights + the same BN vectors, bn_act ops on fp32 tensors (et 2)
    lay32, _ = param_layout(net, "fp32", fold_bn=False)
    assert f"{L.name}.bn_s" in lay32 and lay32[f"{L.name}.w"].dtype == torch.float32
    ops32, _ = build_plan(net, 0, wdtype="fp32", fold_bn=False)
    assert all(op.get("et") == 2 for op in ops32 if op["kind"] == OP_BN_ACT)


def _simulate_chunked(ops, chunk_ops, batch, chunk):
    """Replay the executor's launch order (executor.cpp launch_all) on byte intervals of the
    buffers: every operand read must find, for each of its images, the bytes the op that
    produced it in the unchunked order wrote for that image - nothing overwritten in between."""
    writes = {}  # buffer -> [(lo_byte, hi_byte, writer op, first image, bpi)]

    def write(buf, op_i, i0, n, bpi):
        writes.setdefault(buf, []).append((i0 * bpi, (i0 + n) * bpi, op_i, i0, bpi))

    def check(buf, want, i0, n, bpi):
        for img in range(i0, i0 + n):
            lo, hi = img * bpi, (img + 1) * bpi
            last = next((w for w in reversed(writes.get(buf, [])) if w[0] < hi and lo < w[1]),
                        None)
            assert last is not None and last[2] == want and last[4] == bpi, (buf, want, img)
            assert lo >= last[0] and hi <= last[1]

    # producer of each operand in plain (unchunked) order
    producer, last_writer = [], {0: -1}
    for i, op in enumerate(ops):
        producer.append({k: last_writer.get(op[k]) for k in ("in", "res") if op.get(k, -1) >= 0})
        last_writer[op["out"]] = i

    def run(lo, hi, i0, n):
        for i in range(lo, hi):
            op = ops[i]
            for k, slot in (("in", 0), ("res", 2)):
                if op.get(k, -1) >= 0 and producer[i][k] >= 0:
                    check(op[k], producer[i][k], i0, n, op["bpi"][slot])
            write(op["out"], i, i0, n, op["bpi"][1])

    for c0 in range(0, batch, chunk):
        run(0, chunk_ops, c0, min(chunk, batch - c0))
    run(chunk_ops, len(ops), 0, batch)


@pytest.mark.parametrize("end", ["l1.0.down", "l2.0.down", "l2.0.conv2", "l2.0.conv3",
                                 "l3.0.conv1"])
def test_chunked_plan_keeps_live_out_tensors(end):
    """build_plan(chunk_layers=k): replaying the chunked launch order on buffer byte ranges, no
    chunk overwrites rows another op still reads (live-out tensors of the prefix sit in buffers
    no other prefix tensor uses); the unchunked allocation would fail this."""
    net = get_model("resnet50")
    k = [L.name for L in net.layers].index(end)
    ops, _ = build_plan(net, 0, chunk_layers=k)
    n = sum(1 for op in ops if op["layer"] < k)
    _simulate_chunked(ops, n, batch=7, chunk=3)
    _simulate_chunked(ops, n, batch=6, chunk=3)
    if end in ("l2.0.conv2", "l2.0.conv3"):
        plain, _ = build_plan(net, 0)
        with pytest.raises(AssertionError):
            _simulate_chunked(plain, n, batch=7, chunk=3)


def test_resnet50_plan_fuses_56x56_bottlenecks(monkeypatch):
    """fuse_stem_pool / fuse_bottlenecks: stem conv + max-pool become one OP_STEM_POOL, and the
    three 56x56 blocks (block 0 with its projection) become one
    OP_BOTTLENECK each, wired from the block input to the block output buffer; other stages,
    fp8 and the unfused switch keep the layered ops. (The strided projections of l2-l4 are
    covered by the next test and left out here.)"""
    from gale.models.graph import OP_BOTTLENECK, OP_CONV, OP_STEM_POOL

    monkeypatch.setenv("GALE_FUSE_PROJ", "0")
    net = get_model("resnet50")
    layered, bufs = build_plan(net, 1 << 20, fuse_blocks=False)
    fused, bufs2 = build_plan(net, 1 << 20, fuse_blocks=True)
    assert bufs == bufs2
    bn = [op for op in fused if op["kind"] == OP_BOTTLENECK]
    assert [op["p"][:2] for op in bn] == [[64, 1], [256, 0], [256, 0]]
    assert len(fused) == len(layered) - 4 - 3 - 3 + 3 - 1  # (- 1: stem + max-pool fused)
    sp = [op for op in fused if op["kind"] == OP_STEM_POOL]
    assert len(sp) == 1 and fused[1] is sp[0]
    assert sp[0]["in"] == layered[1]["in"] and sp[0]["out"] == layered[2]["out"]
    assert sp[0]["w"] == layered[1]["w"] and sp[0]["p"] == layered[2]["p"]
    # block 0 reads the max-pool output and writes what l1.1 reads; each block feeds the next
    assert bn[0]["in"] == layered[2]["out"]  # stem_pack, stem, maxpool -> p0
    assert bn[1]["in"] == bn[0]["out"] and bn[2]["in"] == bn[1]["out"]
    assert all(op["in"] != op["out"] for op in bn)
    nxt = fused[fused.index(bn[2]) + 1]
    assert nxt["kind"] == OP_CONV and nxt["in"] == bn[2]["out"]  # l2.0.down reads l1's output
    assert len(bn[0]["ptrs"]) == 8 and len(bn[1]["ptrs"]) == 6
    # pointers are the layered convs' own packed weights / biases
    l1 = [op for op in layered[3:13]]
    assert bn[0]["ptrs"][:6] == [l1[1]["w"], l1[1]["bias"], l1[2]["w"], l1[2]["bias"],
                                 l1[3]["w"], l1[3]["bias"]]
    assert bn[0]["ptrs"][6:] == [l1[0]["w"], l1[0]["bias"]]
    # other models / dtypes untouched
    r20 = build_plan(get_model("resnet20"), 1 << 20, fused=False, fuse_blocks=True)[0]
    assert not any(op["kind"] == OP_BOTTLENECK for op in r20)


def test_stem_pool_not_fused_when_the_stem_output_is_read_again():
    """fuse_stem_pool only fuses when nothing else reads the stem output (it never reaches memory
    in the fused kernel)."""
    from gale.models.graph import (OP_STEM_POOL, AvgPool, Conv, Head, MaxPool, Network,
                                   build_plan)

    def net(extra_reader):
        L = [Conv("stem", "input", "s0", 3, 64, 7, stride=2, pad=3),
             MaxPool("pool", "s0", "p0", 3, 2, 1)]
        if extra_reader:  # a 1x1 conv on the stem output itself
            L.append(Conv("side", "s0", "sd", 64, 64, 1))
            L.append(AvgPool("gp", "sd", "g"))
        else:
            L.append(AvgPool("gp", "p0", "g"))
        L.append(Head("fc", "g", 10))
        return Network("stemtest", (224, 224, 3), 10, L, dataset="imagenet")

    fused = build_plan(net(False), 1 << 20, fuse_blocks=True)[0]
    kept = build_plan(net(True), 1 << 20, fuse_blocks=True)[0]
    assert sum(op["kind"] == OP_STEM_POOL for op in fused) == 1
    assert not any(op["kind"] == OP_STEM_POOL for op in kept)


def test_resnet50_plan_fuses_strided_projections_into_conv3():
    """l2.0 / l3.0 / l4.0: the 1x1/2 projection runs inside conv3 (OP_CONV_PROJ, one GEMM over
    the concatenated reduction); the block input it reads stays in its buffer until then."""
    from gale.models import get_model
    from gale.models.graph import OP_CONV, OP_CONV_PROJ, build_plan

    net = get_model("resnet50")
    ops, _ = build_plan(net, 0, "bf16", fuse_blocks=True)
    layered, _ = build_plan(net, 0, "bf16", fuse_blocks=False)
    proj = [k for k, o in enumerate(ops) if o["kind"] == OP_CONV_PROJ]
    assert len(proj) == 3
    assert len(ops) == len(layered) - 3 - 2 - 3 * 3 + 3  # - projections, stem/pool, l1 blocks
    for k in proj:
        op = ops[k]
        c1, c2 = ops[k - 2], ops[k - 1]
        assert c1["kind"] == c2["kind"] == OP_CONV
        # conv1 reads the block input; neither conv1 nor conv2 overwrites it before conv3
        assert c1["in"] == op["res"] and op["res"] not in (c1["out"], c2["out"])
        assert op["in"] == c2["out"] and op["out"] != op["res"]
        H2, W2, Cin2, s2, Kpad2 = op["p"]
        d = op["conv"]
        assert s2 == 2 and (H2 - 1) // 2 + 1 == d["Ho"] and Kpad2 == Cin2
        assert d["KH"] == 1 and d["stride"] == 1 and not d.get("has_res")
        assert op["bpi"][2] == c1["bpi"][0]
        assert len(op["ptrs"]) == 4
    # no other op reads a projection's (now unwritten) output buffer
    written = {o["out"] for o in ops}
    for o in ops:
        assert o["in"] in written | {0} and o.get("res", -1) in written | {-1, 0}
