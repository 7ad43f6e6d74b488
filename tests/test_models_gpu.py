"""End-to-end model numerics: the gfx950 plan (eager and hipGraph replay) vs the fp32 oracle.

Comparisons are on LOGITS (the softmax inverted: centered log-probabilities, exact up to the
per-row constant the softmax removes), relative to the row's logit scale, so an error that
would hide inside probabilities near 1/classes still fails."""

import pytest
import torch


def logits(p: torch.Tensor) -> torch.Tensor:
    lp = p.double().clamp_min(1e-300).log()
    return lp - lp.mean(dim=1, keepdim=True)


def rel_logit_err(p: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
    """Per-row max |dlogit| / max(|ref logit|, 1)."""
    a, b = logits(p), logits(ref)
    return (a - b).abs().amax(1) / b.abs().amax(1).clamp_min(1.0)


def margin(ref: torch.Tensor) -> torch.Tensor:
    top2 = ref.topk(2, dim=1).values
    return top2[:, 0] - top2[:, 1]

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
    # (the fused LeNet-5 keeps its activations in fp32: only its weights are bf16)
    emu = forward(net, fold_params(net, params), x, bf16=True, bf16_acts=name != "lenet5")
    assert eager.shape == ref.shape
    err = rel_logit_err(eager, ref).max().item()
    e_emu = rel_logit_err(eager, emu).max().item()
    budget = rel_logit_err(emu, ref).max().item()  # what bf16 storage alone costs
    print(f"\n{name} bf16 rel logit err vs fp32 {err:.2e} (bf16 emulation vs fp32 "
          f"{budget:.2e}), vs bf16 emulation {e_emu:.2e}")
    # the kernels match the bf16 emulation up to accumulation order, and are no further from
    # fp32 than bf16 storage itself puts them
    # (deep nets amplify accumulation-order rounding flips: allow a fraction of the budget)
    assert e_emu < max(1e-2, 0.35 * budget), f"{name}: vs bf16 emulation {e_emu}"
    assert err < 1.5 * budget + 5e-3, f"{name}: relative logit error {err} (budget {budget})"
    clear = margin(ref) > 0.05  # argmax must agree wherever it is not a near-tie
    assert torch.equal(eager.argmax(1)[clear], ref.argmax(1)[clear])
    # graph replay (bucket >= batch, padded tail) must equal eager bit for bit; one-kernel plans
    # (the fused ResNet-20) launch directly instead
    assert torch.equal(graph, eager)
    assert (rep.executor.graphs_captured >= 1) == rep.executor.graph_pays


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
    emu = forward(net, fold_params(net, params), x, bf16=True)
    torch.cuda.synchronize()
    e_ab, e_emu = rel_logit_err(a, b).max().item(), rel_logit_err(a, emu).max().item()
    e_ref, budget = rel_logit_err(a, ref).max().item(), rel_logit_err(emu, ref).max().item()
    print(f"\nresnet50 gemm vs mfma {e_ab:.2e}, vs bf16 emulation {e_emu:.2e}, vs fp32 "
          f"{e_ref:.2e} (budget {budget:.2e})")
    assert e_ab < max(1e-2, 0.35 * budget) and e_emu < max(1e-2, 0.35 * budget)
    assert e_ref < 1.5 * budget + 5e-3
    assert torch.allclose(a.sum(1), torch.ones(6), atol=1e-4)


def test_resnet50_fused_projection_vs_layered(monkeypatch):
    """OP_CONV_PROJ (conv3 + the strided projection shortcut as one GEMM, conv2d_gemm_proj)
    against the layered plan (GALE_FUSE_PROJ=0: the projection is its own conv, stored as bf16,
    and conv3 adds it). The fused epilogue adds the projection's fp32 accumulator unrounded
    (conv_gemm.hip DUAL note), so the two agree to accumulation / one bf16 rounding of the
    shortcut - well inside the bf16 budget - and both match the bf16 emulation."""
    net = get_model("resnet50")
    params = init_params(net, seed=31, calib_batch=4)
    packed = materialize_weights(net, torch.device("cuda", 0), params=params)
    x = torch.rand((5,) + net.input_shape, generator=torch.Generator().manual_seed(13))
    monkeypatch.setenv("GALE_FUSE_PROJ", "1")
    fused = ModelReplica(net, packed, max_batch=8, slots=1)
    monkeypatch.setenv("GALE_FUSE_PROJ", "0")
    layered = ModelReplica(net, packed, max_batch=8, slots=1)
    assert sum(op["kind"] == 11 for op in fused.ops) == 3  # l2.0 / l3.0 / l4.0
    assert not any(op["kind"] == 11 for op in layered.ops)
    a = fused.infer_eager(x).cpu()
    b = layered.infer_eager(x).cpu()
    torch.cuda.synchronize()
    folded = fold_params(net, params)
    emu = forward(net, folded, x, bf16=True)
    budget = rel_logit_err(emu, forward(net, folded, x)).max().item()
    e_ab, e_emu = rel_logit_err(a, b).max().item(), rel_logit_err(a, emu).max().item()
    print(f"\nresnet50 fused proj vs layered {e_ab:.2e}, vs bf16 emulation {e_emu:.2e} "
          f"(budget {budget:.2e})")
    assert e_ab < max(1e-2, 0.35 * budget) and e_emu < max(1e-2, 0.35 * budget)


@pytest.mark.parametrize("end", ["l2.0.down", "l2.0.conv3"])
def test_resnet50_batch_chunked_prefix_is_bit_identical(end, monkeypatch):
    """PlanSpec chunking (the leading layers run per chunk of images, the rest over the whole
    batch) changes only the launch grids: every output element keeps its kernel and k-order, so
    logits are bit identical to the unchunked plan, eager and graph, with a ragged last chunk.
    "l2.0.conv3": the prefix ends mid-block, its live-out shortcut (l2.0.down) is produced
    before the last prefix op and must survive the later chunks. (A chunked plan keeps the
    projections as separate convs, so the unchunked one does too here: fused into conv3 the
    shortcut is no longer rounded to bf16 before the add.)"""
    monkeypatch.setenv("GALE_FUSE_PROJ", "0")
    net = get_model("resnet50")
    params = init_params(net, seed=23, calib_batch=4)
    packed = materialize_weights(net, torch.device("cuda", 0), params=params)
    x = torch.rand((7,) + net.input_shape, generator=torch.Generator().manual_seed(9))
    n_pre = [L.name for L in net.layers].index(end)
    base = ModelReplica(net, packed, max_batch=8, slots=1)
    chunked = ModelReplica(net, packed, max_batch=8, slots=1, chunk=(n_pre, 3))
    a = base.infer_eager(x).cpu()
    b = chunked.infer_eager(x).cpu()
    c = chunked.infer(x).cpu()
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(a, c)


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
    e_emu = rel_logit_err(got, emu)
    e_ref = rel_logit_err(got, ref)
    budget = rel_logit_err(emu, ref)  # what e4m3 quantisation alone costs
    print(f"\n{name} fp8 vs emulation mean {e_emu.mean().item():.2e} max "
          f"{e_emu.max().item():.2e}; vs fp32 mean {e_ref.mean().item():.2e} max "
          f"{e_ref.max().item():.2e} (quantisation budget mean {budget.mean().item():.2e})")
    # e4m3 rounding flips (fp32 summation order) compound with depth: ResNet-50's 53 layers
    # decorrelate kernel and emulation up to the quantisation budget itself
    frac = 1.0 if name == "resnet50" else 0.5
    assert e_emu.mean().item() < max(1e-2, frac * budget.mean().item()), \
        f"{name}: fp8 vs emulation {e_emu.mean().item()}"
    # the kernels are no further from fp32 than the quantisation itself puts them
    assert e_ref.mean().item() < 1.25 * budget.mean().item() + 5e-3
    clear = margin(ref) > 0.05
    if clear.any():  # (1000-class random-init resnet50 has no clear winner)
        agree = (got.argmax(1)[clear] == ref.argmax(1)[clear]).float().mean().item()
        assert agree >= 0.97, f"{name}: fp8 argmax agreement {agree}"


@pytest.mark.parametrize("batch", [1, 13, 257, 1000])
def test_lenet5_fused_matches_layerwise_and_fp32(batch):
    """The whole-network LeNet-5 kernel (one image per workgroup, fp32 activations in LDS, bf16
    weights) against the layer-by-layer bf16 plan on the same packed weights, the weight-only
    bf16 emulation (tight: same operands, fp32 everywhere else) and the fp32 oracle, at batches
    across graph buckets."""
    net = get_model("lenet5")
    params = init_params(net, seed=19)
    packed = materialize_weights(net, torch.device("cuda", 0), params=params)
    fused = ModelReplica(net, packed, max_batch=1024, slots=1, fused=True)
    layered = ModelReplica(net, packed, max_batch=1024, slots=1, fused=False)
    assert len(fused.ops) == 1 and len(layered.ops) > 1
    x = torch.rand((batch, 28, 28, 1), generator=torch.Generator().manual_seed(batch))
    a = fused.infer(x, use_graph=True).cpu()
    b = layered.infer(x, use_graph=True).cpu()
    folded = fold_params(net, params)
    ref = forward(net, folded, x)
    emu_w = forward(net, folded, x, bf16=True, bf16_acts=False)
    emu = forward(net, folded, x, bf16=True)
    torch.cuda.synchronize()
    e_w = rel_logit_err(a, emu_w).max().item()
    e_ab, e_ref = rel_logit_err(a, b).max().item(), rel_logit_err(a, ref).max().item()
    budget = rel_logit_err(emu, ref).max().item()
    print(f"\nlenet5 fused vs weight-bf16 emulation {e_w:.2e}, vs layered {e_ab:.2e}, vs fp32 "
          f"{e_ref:.2e} (bf16 budget {budget:.2e})")
    assert e_w < 1e-4  # fp32 math on the same bf16 weights: summation order only
    assert e_ab < 1.5 * budget + 5e-3 and e_ref < 1.5 * budget + 5e-3
    assert torch.allclose(a.sum(1), torch.ones(batch), atol=1e-5)
    assert torch.equal(fused.infer_eager(x).cpu(), a)


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
    emu = forward(net, fold_params(net, params), x, bf16=True)
    torch.cuda.synchronize()
    e_ab, e_emu = rel_logit_err(a, b).max().item(), rel_logit_err(a, emu).max().item()
    e_ref, budget = rel_logit_err(a, ref).max().item(), rel_logit_err(emu, ref).max().item()
    print(f"\nresnet20 fused vs layered {e_ab:.2e}, vs bf16 emulation {e_emu:.2e}, vs fp32 "
          f"{e_ref:.2e} (budget {budget:.2e})")
    assert e_ab < 5e-3 and e_emu < 5e-3 and e_ref < 1.5 * budget + 5e-3
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
    budget = rel_logit_err(emu, forward(net, fold_params(net, params), x)).mean().item()
    e_ab, e_emu = rel_logit_err(a, b).mean().item(), rel_logit_err(a, emu).mean().item()
    print(f"\nresnet20 fp8 fused vs layered mean {e_ab:.2e}, vs emulation {e_emu:.2e} "
          f"(quantisation budget {budget:.2e})")
    assert e_ab < 1e-3 and e_emu < 0.5 * budget
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
    budget = rel_logit_err(forward(net, fold_params(net, params), x, bf16=True), ref).max().item()
    eager = rep.infer_eager(x).cpu()
    graph = rep.infer(x, use_graph=True).cpu()
    torch.cuda.synchronize()
    err = rel_logit_err(eager, ref).max().item()
    print(f"\n{name} unfolded-BN rel logit err {err:.2e} (budget {budget:.2e})")
    # one more bf16 rounding point than the folded plan (the raw conv output before BN)
    assert err < 2 * budget + 1e-2, f"{name}: relative logit error {err}"
    clear = margin(ref) > 0.05
    assert torch.equal(eager.argmax(1)[clear], ref.argmax(1)[clear])
    assert torch.equal(graph, eager)


@pytest.mark.parametrize("name,batch", [("resnet20", 19), ("resnet50", 2)])
def test_fp32_unfolded_bn_plan_matches_reference(name, batch):
    """--dtype fp32 --no-fold-bn: raw fp32 convs, then the standalone BatchNorm(+residual+ReLU)
    kernel on fp32 NHWC (TF's Conv2D -> FusedBatchNorm with no extra rounding point): relative
    logit error < 1e-4 against the fp32 oracle."""
    from gale.models.graph import OP_BN_ACT

    net = get_model(name)
    params = init_params(net, seed=23, calib_batch=4 if name == "resnet50" else 16)
    packed = materialize_weights(net, torch.device("cuda", 0), params=params, wdtype="fp32",
                                 fold_bn=False)
    rep = ModelReplica(net, packed, max_batch=32, slots=1, wdtype="fp32", fold_bn=False)
    assert sum(op["kind"] == OP_BN_ACT for op in rep.ops) > 0
    x = torch.rand((batch,) + net.input_shape, generator=torch.Generator().manual_seed(6))
    ref = forward(net, fold_params(net, params), x)
    got = rep.infer(x, use_graph=True).cpu()
    torch.cuda.synchronize()
    err = rel_logit_err(got, ref).max().item()
    print(f"\n{name} fp32 unfolded-BN rel logit err {err:.2e}")
    assert err < 1e-4, err
    assert torch.equal(got.argmax(1), ref.argmax(1))


@pytest.mark.parametrize("name,batch", [("lenet5", 13), ("resnet20", 37), ("resnet50", 3)])
def test_fp32_plan_matches_fp32_reference(name, batch):
    """--dtype fp32: the reference-precision plan (fp32 weights and activations, convs on the fp32
    matrix core v_mfma_f32_16x16x4_f32) agrees with the fp32 oracle to summation order: relative
    logit error < 1e-4, argmax identical, eager == graph replay."""
    net = get_model(name)
    params = init_params(net, seed=11, calib_batch=4 if name == "resnet50" else 16)
    packed = materialize_weights(net, torch.device("cuda", 0), params=params, wdtype="fp32")
    rep = ModelReplica(net, packed, max_batch=64, slots=1, wdtype="fp32")
    assert all(op["conv"]["f32"] == 1 for op in rep.ops if op["kind"] == 0)
    x = torch.rand((batch,) + net.input_shape, generator=torch.Generator().manual_seed(99))
    ref = forward(net, fold_params(net, params), x)
    eager = rep.infer_eager(x).cpu()
    graph = rep.infer(x, use_graph=True).cpu()
    torch.cuda.synchronize()
    err = rel_logit_err(eager, ref).max().item()
    print(f"\n{name} fp32 plan rel logit err {err:.2e}")
    assert err < 1e-4, f"{name}: fp32 plan relative logit error {err}"
    assert torch.equal(eager.argmax(1), ref.argmax(1))
    assert torch.equal(graph, eager)
