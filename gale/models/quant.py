"""OCP fp8 (e4m3fn) quantisation for the fp8 serving path (BASELINE.json config 5).

gfx950 MFMA consumes OCP ``e4m3fn`` (bias 7, max 448, no infinities) — not the MI300 ``fnuz``
variant (``/opt/skills/guides/cdna_hip_programming.md`` §4) — which is exactly torch's
``torch.float8_e4m3fn``, so host-side packing and the emulation oracle use torch's casts.

* weights: per-output-channel scale, ``w = code * s[c]`` with ``s[c] = amax_c / 448``;
* activations: one scale per tensor, calibrated offline from the fp32 oracle on synthetic
  inputs of the serving distribution (``calibrate_act_scales``); the network input stays fp32 on
  the wire and is quantised by the stem while it is loaded.

The reference has no reduced-precision path (TF-Java CPU fp32, InferenceBolt.java:80-86); fp8 is
a new capability whose accuracy is pinned against the fp32 oracle by the tests.
"""

from __future__ import annotations

from typing import Dict, Tuple

import torch

E4M3_MAX = 448.0
CALIB_SEED = 4321
CALIB_BATCH = 64
CALIB_MARGIN = 1.25  # headroom over the calibration amax (unseen inputs of the same distribution)


def e4m3_round(x: torch.Tensor) -> torch.Tensor:
    """Round fp32 values to the nearest e4m3 value (saturating at +-448)."""
    return x.clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn).float()


def e4m3_codes(x: torch.Tensor) -> torch.Tensor:
    return x.clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn).view(torch.uint8)


def quantize_rows_e4m3(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """[N, K] fp32 -> (uint8 e4m3 codes [N, K], fp32 per-row scales [N]); w ~= code * s[row]."""
    amax = w.abs().amax(dim=1)
    s = torch.where(amax > 0, amax / E4M3_MAX, torch.ones_like(amax))
    return e4m3_codes(w / s[:, None]), s.float().contiguous()


def dequantize_rows_e4m3(q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    return q.view(torch.float8_e4m3fn).float() * s[:, None]


def fake_quant_weight(w: torch.Tensor) -> torch.Tensor:
    """[cout, cin, kh, kw] -> the fp32 weight the fp8 kernel effectively uses."""
    flat = w.reshape(w.shape[0], -1)
    q, s = quantize_rows_e4m3(flat)
    return dequantize_rows_e4m3(q, s).reshape(w.shape)


def activation_tensors(net) -> list:
    """Names of every activation tensor that gets an fp8 scale: the input, then each producer."""
    from gale.models.graph import AvgPool, Conv, MaxPool

    names = ["input"]
    for L in net.layers:
        if isinstance(L, (Conv, MaxPool, AvgPool)):
            names.append(L.out)
    return names


@torch.no_grad()
def calibrate_act_scales(net, folded: Dict[str, torch.Tensor]) -> Dict[str, float]:
    """Per-tensor e4m3 scales from the fp32 oracle on a seeded U[0,1) calibration batch.

    Pooling outputs inherit their input's scale (max / mean never leave its range), so pool ops
    pass codes through unchanged.
    """
    from gale.models.graph import AvgPool, MaxPool
    from gale.models.reference import forward

    g = torch.Generator().manual_seed(CALIB_SEED)
    x = torch.rand((CALIB_BATCH,) + tuple(net.input_shape), generator=g)
    tensors: Dict[str, torch.Tensor] = {}
    forward(net, folded, x, tensors=tensors)
    scales: Dict[str, float] = {}
    for name in activation_tensors(net):
        amax = float(tensors[name].abs().max())
        scales[name] = max(amax * CALIB_MARGIN, 1e-6) / E4M3_MAX
    for L in net.layers:
        if isinstance(L, (MaxPool, AvgPool)):
            scales[L.out] = scales[L.inp]
    return scales
