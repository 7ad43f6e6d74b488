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
    assert len(buf_bytes) <= 6


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
