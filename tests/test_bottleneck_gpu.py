"""The fused ResNet-50 kernels against the layered kernels they replace: the 56x56 bottleneck
(csrc/kernels/bottleneck_fused.hip; also against a PyTorch fp32 oracle of the block), the stem +
max-pool (csrc/kernels/stem_pool.hip), and the whole ResNet-50 forward with and without the
fusions (gale.models.graph.fuse_stem_pool / fuse_bottlenecks)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _weights(g, cin, down):
    def conv(cout, ci, k):
        w = torch.randn(cout, ci, k, k, generator=g) * (2.0 / (k * k * ci)) ** 0.5
        b = torch.randn(cout, generator=g) * 0.1
        return w, b
    ws = {"c1": conv(64, cin, 1), "c2": conv(64, 64, 3), "c3": conv(256, 64, 1)}
    if down:
        ws["d"] = conv(256, cin, 1)
    return ws


def _bf(t):
    return t.to(torch.bfloat16).float()


def _oracle(x, ws, down):
    """fp32 block with bf16 rounding where the kernels store bf16 tensors (NCHW math)."""
    xn = x.permute(0, 3, 1, 2)

    def conv(t, key, pad, relu):
        w, b = ws[key]
        y = F.conv2d(t, _bf(w), b, padding=pad)
        return torch.relu(y) if relu else y

    a = _bf(conv(xn, "c1", 0, True))
    h = _bf(conv(a, "c2", 1, True))
    sc = _bf(conv(xn, "d", 0, False)) if down else xn
    return torch.relu(conv(h, "c3", 0, False) + sc).permute(0, 2, 3, 1)


@pytest.mark.parametrize("down,batch", [(False, 3), (True, 2)])
def test_bottleneck56_matches_layered_and_oracle(down, batch):
    from gale import ops

    cin = 64 if down else 256
    g = torch.Generator().manual_seed(11 + int(down))
    x = _bf(torch.randn(batch, 56, 56, cin, generator=g))
    ws = _weights(g, cin, down)
    packed = {k: ops.pack_conv(w, b, device=DEV) for k, (w, b) in ws.items()}
    xd = x.to(DEV, torch.bfloat16)

    # layered plan: conv1, conv2 (3x3), [projection], conv3 + shortcut
    (w1, b1, g1), (w2, b2, g2), (w3, b3, g3) = packed["c1"], packed["c2"], packed["c3"]
    a = ops.conv2d(xd, w1, b1, g1, relu=True)
    h = ops.conv2d(a, w2, b2, g2, pad=1, relu=True)
    if down:
        wd, bd, gd = packed["d"]
        sc = ops.conv2d(xd, wd, bd, gd, relu=False)
    else:
        sc = xd
    ref_layered = ops.conv2d(h, w3, b3, g3, relu=True, residual=sc)

    fused = ops.bottleneck56(xd, w1, b1, w2, b2, w3, b3,
                             packed["d"][0] if down else None, packed["d"][1] if down else None)
    torch.cuda.synchronize()
    got, lay = fused.float().cpu(), ref_layered.float().cpu()
    # same bf16 rounding points; only the fp32 accumulation order differs: at most a few
    # elements one bf16 ulp apart
    diff = (got - lay).abs()
    scale = lay.abs().max().item()
    assert diff.max().item() <= 2 ** -6 * max(scale, 1.0), diff.max().item()
    assert (diff > 0).float().mean().item() < 0.02
    # against the fp32 oracle (bf16 operands): the layered kernels' own budget
    ref = _oracle(x, ws, down)
    err = (got - ref).abs().max().item()
    assert err < 2e-2 * max(ref.abs().max().item(), 1.0), err
    # every pixel row written (no uninitialised strip / channel)
    assert torch.isfinite(got).all()


def test_bottleneck56_rejects_other_shapes():
    from gale import ops

    x = torch.zeros(1, 28, 28, 256, device=DEV, dtype=torch.bfloat16)
    w = torch.zeros(64, 256, device=DEV, dtype=torch.bfloat16)
    b = torch.zeros(64, device=DEV)
    with pytest.raises(ValueError):
        ops.bottleneck56(x, w, b, w, b, w, b)


def test_resnet50_fused_blocks_match_layered_plan():
    from gale.models import get_model
    from gale.models.graph import OP_BOTTLENECK
    from gale.parallel.weights import materialize_weights
    from gale.runtime.replica import ModelReplica

    net = get_model("resnet50")
    packed = materialize_weights(net, DEV, wdtype="bf16")
    fused = ModelReplica(net, packed, max_batch=4, slots=1, buckets=[4], fuse_blocks=True)
    layered = ModelReplica(net, packed, max_batch=4, slots=1, buckets=[4], fuse_blocks=False)
    assert sum(op["kind"] == OP_BOTTLENECK for op in fused.ops) == 3
    assert not any(op["kind"] == OP_BOTTLENECK for op in layered.ops)
    g = torch.Generator().manual_seed(5)
    x = torch.rand(3, 224, 224, 3, generator=g)
    pf = fused.infer(x).cpu()
    pl = layered.infer(x).cpu()
    torch.cuda.synchronize()
    assert torch.allclose(pf.sum(1), torch.ones(3), atol=1e-4)
    assert (pf - pl).abs().max().item() < 2e-3
    assert torch.equal(pf.argmax(1), pl.argmax(1))


def test_stem_pool_matches_layered_stem_and_maxpool():
    """stem_pool.hip (ResNet-50 stem conv + 3x3/2 max-pool in one kernel) against the layered
    packed-stem conv_gemm + maxpool kernels on the model's own packed weights: the same fp32
    accumulation order, so the pooled tensors agree bit for bit (up to a stray rounding)."""
    from gale._native import native
    from gale.models import get_model
    from gale.models.graph import OP_CONV, OP_MAXPOOL, OP_STEM_PACK, build_plan
    from gale.parallel.weights import materialize_weights

    C = native()
    net = get_model("resnet50")
    packed = materialize_weights(net, DEV, wdtype="bf16")
    ops, _ = build_plan(net, packed.data_ptr(), "bf16", fuse_blocks=False)
    pk, st, mp = ops[0], ops[1], ops[2]
    assert (pk["kind"], st["kind"], mp["kind"]) == (OP_STEM_PACK, OP_CONV, OP_MAXPOOL)
    B = 3
    g = torch.Generator().manual_seed(3)
    x = torch.rand(B, 224, 224, 3, generator=g).to(DEV)
    s = torch.cuda.current_stream().cuda_stream
    H, W, Cc, Wp, lp = pk["p"][:5]
    xp = torch.empty(B, 224, Wp, 4, device=DEV, dtype=torch.bfloat16)
    C.stem_pack(B, H, W, Cc, Wp, lp, x.data_ptr(), xp.data_ptr(), s)
    s0 = torch.empty(B, 112, 112, 64, device=DEV, dtype=torch.bfloat16)
    C.conv2d(st["conv"], B, xp.data_ptr(), st["w"], st["bias"], 0, 0, s0.data_ptr(), s)
    ref = torch.empty(B, 56, 56, 64, device=DEV, dtype=torch.bfloat16)
    C.maxpool2d(B, *mp["p"], s0.data_ptr(), ref.data_ptr(), s)
    got = torch.full_like(ref, float("nan"))
    C.stem_pool(B, xp.data_ptr(), st["w"], st["bias"], got.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.isfinite(got.float()).all()
    d = (got.float() - ref.float()).abs()
    assert (d > 0).float().mean().item() < 1e-3
    assert d.max().item() <= 2 ** -7 * max(ref.float().abs().max().item(), 1.0)
