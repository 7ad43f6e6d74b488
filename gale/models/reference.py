"""Plain-PyTorch fp32 forward of a gale ``Network``: the numerics oracle for the HIP path.

Used by tests (kernel / model numerics against the gfx950 kernels) and by ``init_params`` for
BatchNorm calibration. It is never a serving backend ("torch-CPU oracle ... tests
only"). Input is NHWC fp32 as in the InstObj contract; output is the softmax (the reference's
``output/Softmax:0``, InferenceBolt.java:83).
"""

from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

from gale.models.graph import BN_EPS, AvgPool, Conv, Head, MaxPool, Network, Softmax


def _residual(t: torch.Tensor, L: Conv, cout: int) -> torch.Tensor:
    if L.res_mode == "pad":  # option A: stride-2 subsample + zero channel padding
        t = t[:, :, ::2, ::2]
        if t.shape[1] < cout:
            t = F.pad(t, (0, 0, 0, 0, 0, cout - t.shape[1]))
    return t


def forward(net: Network, params: Dict[str, torch.Tensor], x_nhwc: torch.Tensor,
            folded: bool = True, bn_stats: Dict[str, torch.Tensor] | None = None,
            collect: Dict[str, torch.Tensor] | None = None,
            tensors: Dict[str, torch.Tensor] | None = None,
            fp8_scales: Dict[str, float] | None = None,
            bf16: bool = False, bf16_acts: bool = True) -> torch.Tensor:
    """fp32 forward. ``folded``: params come from ``fold_params`` (conv bias already has BN).

    With ``folded=False`` BatchNorm is applied from its running statistics (or, when ``bn_stats``
    is a dict, from batch statistics that are written into it — calibration mode). ``tensors``
    receives every activation (NCHW). ``fp8_scales`` turns this into the emulation of the fp8
    kernel path: e4m3 per-channel weights and every activation rounded to e4m3 at its scale.
    ``bf16`` emulates the bf16 kernel path: conv weights and the network input rounded to bf16,
    every stored activation rounded to bf16 (fp32 accumulation, fp32 bias and head), so the
    kernels can be held to accumulation-order differences against it. ``bf16_acts=False``
    rounds only the conv weights (the fused LeNet-5 kernel: bf16 weights, fp32 input and
    activations).
    """
    if fp8_scales is not None:
        from gale.models.quant import e4m3_round, fake_quant_weight

        def q(name, v):
            s = fp8_scales[name]
            return e4m3_round(v / s) * s
    def rb(v):  # round to bf16 and back
        return v.to(torch.bfloat16).float() if bf16 and bf16_acts else v

    def rw(v):
        return v.to(torch.bfloat16).float() if bf16 else v

    x0 = x_nhwc.float().permute(0, 3, 1, 2)
    t: Dict[str, torch.Tensor] = {"input": q("input", x0) if fp8_scales is not None
                                  else rb(x0)}
    out = None
    for L in net.layers:
        if isinstance(L, Conv):
            w = params[f"{L.name}.weight"]
            if fp8_scales is not None:
                w = fake_quant_weight(w)
            w = rw(w)
            b = params.get(f"{L.name}.bias")
            y = F.conv2d(t[L.inp], w, b, stride=L.stride, padding=L.pad)
            if not folded and L.bn:
                if bn_stats is not None:
                    mean = y.mean(dim=(0, 2, 3))
                    var = y.var(dim=(0, 2, 3), unbiased=False)
                    bn_stats[f"{L.name}.bn.mean"] = mean
                    bn_stats[f"{L.name}.bn.var"] = var
                else:
                    mean = params[f"{L.name}.bn.mean"]
                    var = params[f"{L.name}.bn.var"]
                y = F.batch_norm(y, mean, var, params[f"{L.name}.bn.gamma"],
                                 params[f"{L.name}.bn.beta"], training=False, eps=BN_EPS)
            if L.residual is not None:
                y = y + _residual(t[L.residual], L, L.cout)
            if L.relu:
                y = F.relu(y)
            if fp8_scales is not None and not L.out_f32:
                y = q(L.out, y)
            if not L.out_f32:
                y = rb(y)
            t[L.out] = y
        elif isinstance(L, MaxPool):
            t[L.out] = F.max_pool2d(t[L.inp], L.k, L.s, L.p)
        elif isinstance(L, AvgPool):
            t[L.out] = rb(t[L.inp].mean(dim=(2, 3), keepdim=True))
            if fp8_scales is not None:
                t[L.out] = q(L.out, t[L.out])
        elif isinstance(L, Head):
            pooled = t[L.inp].mean(dim=(2, 3))
            logits = pooled @ params[f"{L.name}.weight"].t() + params[f"{L.name}.bias"]
            if collect is not None:
                collect["logits"] = logits
            out = torch.softmax(logits, dim=1)
        elif isinstance(L, Softmax):
            logits = t[L.inp].flatten(1)[:, : L.classes]
            if collect is not None:
                collect["logits"] = logits
            out = torch.softmax(logits, dim=1)
    assert out is not None, "network has no softmax output"
    if tensors is not None:
        tensors.update(t)
    return out


@torch.no_grad()
def calibrate_bn(net: Network, params: Dict[str, torch.Tensor], x_nhwc: torch.Tensor) -> None:
    """Set every BN's running stats to the batch stats of a synthetic calibration batch."""
    stats: Dict[str, torch.Tensor] = {}
    forward(net, params, x_nhwc, folded=False, bn_stats=stats)
    params.update({k: v.detach().clone() for k, v in stats.items()})
