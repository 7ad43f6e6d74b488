"""End-to-end model numerics: the gfx950 plan (eager and hipGraph replay) vs the fp32 oracle."""

import pytest
import torch

from gale.models import fold_params, get_model, init_params
from gale.models.reference import forward
from gale.parallel.weights import materialize_weights
from gale.runtime.replica import ModelReplica

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,batch", [("lenet5", 13), ("resnet20", 37), ("resnet50", 3)])
def test_model_matches_reference(name, batch):
    net = get_model(name)
    params = init_params(net, seed=11, calib_batch=4 if name == "resnet50" else 16)
    packed = materialize_weights(net, torch.device("cuda", 0), params=params)
    rep = ModelReplica(net, packed, max_batch=64, slots=2)
    g = torch.Generator().manual_seed(99)
    x = torch.rand((batch,) + net.input_shape, generator=g)
    ref = forward(net, fold_params(net, params), x)
    eager = rep.infer_eager(x).cpu()
    graph = rep.infer(x, use_graph=True, slot=1).cpu()
    torch.cuda.synchronize()
    assert eager.shape == ref.shape
    err = (eager - ref).abs().max().item()
    assert err < 3e-2, f"{name}: max |p - p_ref| = {err}"
    top2 = ref.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 0.05  # argmax must agree wherever it is not a near-tie
    assert torch.equal(eager.argmax(1)[clear], ref.argmax(1)[clear])
    # graph replay (bucket >= batch, padded tail) must equal eager bit for bit
    assert torch.equal(graph, eager)
    assert rep.executor.graphs_captured >= 1


def test_resnet50_gemm_convs_match_conv_mfma_and_fp32():
    """ResNet-50 with every wide conv on the LDS-pipelined GEMM kernel and the packed stem
    (conv_gemm.hip) against the same plan on conv_mfma only (the stem stays packed: its layout
    is fixed by the plan) and against the fp32 oracle."""
    from gale._native import native

    net = get_model("resnet50")
    params = init_params(net, seed=21, calib_batch=4)
    packed = materialize_weights(net, torch.device("cuda", 0), params=params)
    rep = ModelReplica(net, packed, max_batch=16, slots=1)
    assert any(op["kind"] == 6 for op in rep.ops)  # OP_STEM_PACK
    x = torch.rand((6,) + net.input_shape, generator=torch.Generator().manual_seed(5))
    C = native()
    try:
        C.set_conv_path(2)
        a = rep.infer_eager(x).cpu()
        C.set_conv_path(1)
        b = rep.infer_eager(x).cpu()
    finally:
        C.set_conv_path(0)
    ref = forward(net, fold_params(net, params), x)
    torch.cuda.synchronize()
    assert (a - b).abs().max().item() < 1e-2
    assert (a - ref).abs().max().item() < 3e-2
    assert torch.allclose(a.sum(1), torch.ones(6), atol=1e-4)


@pytest.mark.parametrize("name,batch", [("lenet5", 13), ("resnet20", 37), ("resnet50", 2)])
def test_fp8_model_matches_emulation_and_fp32(name, batch):
    """fp8 plan (e4m3 MFMA, calibrated per-tensor activation scales) against the fp8 emulation
    oracle (tight: same quantised operands) and against the fp32 oracle (accuracy budget)."""
    from gale.models.graph import act_scales_from_packed

    net = get_model(name)
    params = init_params(net, seed=11, calib_batch=4 if name == "resnet50" else 16)
    packed = materialize_weights(net, torch.device("cuda", 0), params=params, wdtype="fp8")
    rep = ModelReplica(net, packed, max_batch=64, slots=1, wdtype="fp8")
    x = torch.rand((batch,) + net.input_shape, generator=torch.Generator().manual_seed(99))
    folded = fold_params(net, params)
    emu = forward(net, folded, x, fp8_scales=act_scales_from_packed(net, packed))
    ref = forward(net, folded, x)
    got = rep.infer(x, use_graph=True).cpu()
    torch.cuda.synchronize()
    e_emu = (got - emu).abs()
    assert e_emu.mean().item() < 5e-3, f"{name}: mean |p - p_emu| = {e_emu.mean().item()}"
    e_ref = (got - ref).abs()
    assert e_ref.max().item() < 0.2 and e_ref.mean().item() < 0.02
    top2 = ref.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 0.1
    if clear.any():  # (1000-class random-init resnet50 has no clear winner)
        assert (got.argmax(1)[clear] == ref.argmax(1)[clear]).float().mean().item() >= 0.9


@pytest.mark.parametrize("batch", [1, 37, 600])
def test_resnet20_fused_matches_layerwise_and_fp32(batch):
    """The whole-network fused kernel (activations in LDS, persistent over images) against the
    layer-by-layer plan on the same packed weights and against the fp32 oracle. batch 600 >
    2 workgroups x 256 CUs exercises the grid-stride image loop."""
    net = get_model("resnet20")
    params = init_params(net, seed=17)
    packed = materialize_weights(net, torch.device("cuda", 0), params=params)
    fused = ModelReplica(net, packed, max_batch=600, slots=1, fused=True)
    layered = ModelReplica(net, packed, max_batch=600, slots=1, fused=False)
    assert len(fused.ops) == 1 and len(layered.ops) > 1
    x = torch.rand((batch, 32, 32, 3), generator=torch.Generator().manual_seed(batch))
    a = fused.infer(x, use_graph=True).cpu()
    b = layered.infer(x, use_graph=True).cpu()
    ref = forward(net, fold_params(net, params), x)
    torch.cuda.synchronize()
    assert (a - b).abs().max().item() < 2e-3
    assert (a - ref).abs().max().item() < 3e-2
    assert torch.allclose(a.sum(1), torch.ones(batch), atol=1e-5)
    # eager launch equals graph replay
    assert torch.equal(fused.infer_eager(x).cpu(), a)


def test_resnet20_fp8_fused_matches_layerwise():
    """fp8 whole-network kernel (e4m3 activations in LDS) against the per-layer fp8 plan and the
    fp8 emulation oracle on the same packed weights / calibrated scales."""
    from gale.models.graph import act_scales_from_packed

    net = get_model("resnet20")
    params = init_params(net, seed=5)
    packed = materialize_weights(net, torch.device("cuda", 0), params=params, wdtype="fp8")
    fused = ModelReplica(net, packed, max_batch=700, slots=1, wdtype="fp8", fused=True)
    layered = ModelReplica(net, packed, max_batch=700, slots=1, wdtype="fp8", fused=False)
    assert len(fused.ops) == 1 and len(layered.ops) > 1
    x = torch.rand((700, 32, 32, 3), generator=torch.Generator().manual_seed(3))
    a = fused.infer(x, use_graph=True).cpu()
    b = layered.infer(x, use_graph=True).cpu()
    emu = forward(net, fold_params(net, params), x, fp8_scales=act_scales_from_packed(net, packed))
    torch.cuda.synchronize()
    # same quantised operands and rounding points; only fp32 summation order differs, which can
    # flip an occasional e4m3 rounding
    assert (a - b).abs().mean().item() < 2e-3
    assert (a - emu).abs().mean().item() < 5e-3
    assert (a.argmax(1) == b.argmax(1)).float().mean().item() > 0.97


@pytest.mark.parametrize("name,batch", [("resnet20", 21), ("resnet50", 2)])
def test_unfolded_bn_plan_matches_reference(name, batch):
    """The debugging / parity plan: raw convs + standalone BatchNorm(+residual+ReLU) kernels
    against the fp32 oracle, eager and graph replay."""
    from gale.models.graph import OP_BN_ACT

    net = get_model(name)
    params = init_params(net, seed=17, calib_batch=4 if name == "resnet50" else 16)
    packed = materialize_weights(net, torch.device("cuda", 0), params=params, fold_bn=False)
    rep = ModelReplica(net, packed, max_batch=32, slots=1, fold_bn=False)
    assert sum(op["kind"] == OP_BN_ACT for op in rep.ops) > 0
    x = torch.rand((batch,) + net.input_shape, generator=torch.Generator().manual_seed(4))
    ref = forward(net, fold_params(net, params), x)
    eager = rep.infer_eager(x).cpu()
    graph = rep.infer(x, use_graph=True).cpu()
    torch.cuda.synchronize()
    err = (eager - ref).abs().max().item()
    assert err < 4e-2, f"{name}: max |p - p_ref| = {err}"
    top2 = ref.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 0.05
    assert torch.equal(eager.argmax(1)[clear], ref.argmax(1)[clear])
    assert torch.equal(graph, eager)
