"""PyTorch-facing wrappers of the gale gfx950 kernels (``gale._C``).

Each op takes device tensors, launches the hand-written HIP kernel on the current torch stream
and returns a new tensor. There is deliberately no eager-PyTorch fallback: if the native library
is missing or the tensor is not on a GPU the call fails loudly (the serving path must never run
silently on a non-native implementation).
"""

from __future__ import annotations

from typing import Optional

import torch

from gale._native import native
from gale.models.graph import conv_n_tiles, pack_conv_weight, round_up


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _check(t: torch.Tensor, dtype: torch.dtype, name: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"gale op: {name} must be a GPU tensor (no CPU fallback)")
    if t.dtype != dtype:
        raise TypeError(f"gale op: {name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"gale op: {name} must be contiguous")


def pack_conv(w_oihw: torch.Tensor, bias: torch.Tensor, cin_stored: Optional[int] = None,
              device=None):
    """Pack an fp32 [Cout, Cin, KH, KW] conv weight for the MFMA kernel.

    Returns (w_packed bf16 [Npad, Kpad], bias fp32 [Npad], desc-geometry dict).
    """
    cout, cin, kh, kw = w_oihw.shape
    cin_s = cin if cin_stored is None else cin_stored
    cout_s = round_up(cout, 4)
    K = kh * kw * cin_s
    Kpad = round_up(K, 32)
    Npad = round_up(cout_s, conv_n_tiles(cout_s) * 16)
    wp = pack_conv_weight(w_oihw.float().cpu(), cin_s, Npad, Kpad).to(torch.bfloat16)
    bp = torch.zeros(Npad)
    bp[:cout] = bias.float().cpu()
    dev = device if device is not None else torch.device("cuda")
    return wp.to(dev), bp.to(dev), dict(Cin=cin_s, Cout=cout_s, KH=kh, KW=kw, K=K, Kpad=Kpad,
                                        Npad=Npad)


def conv2d(x: torch.Tensor, w_packed: torch.Tensor, bias: torch.Tensor, geom: dict, stride: int = 1,
           pad: int = 0, relu: bool = False, residual: Optional[torch.Tensor] = None,
           res_mode: str = "identity", out_f32: bool = False) -> torch.Tensor:
    """NHWC conv on MFMA. x: [B,H,W,Cin] bf16 (or fp32 for the network input)."""
    B, H, W, C = x.shape
    if C != geom["Cin"]:
        raise ValueError(f"x has {C} channels, packed weight expects {geom['Cin']}")
    _check(w_packed, torch.bfloat16, "w_packed")
    _check(bias, torch.float32, "bias")
    if x.dtype not in (torch.bfloat16, torch.float32):
        raise TypeError("x must be bf16 or fp32")
    _check(x, x.dtype, "x")
    kh, kw = geom["KH"], geom["KW"]
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    cout = geom["Cout"]
    y = torch.empty(B, Ho, Wo, cout, device=x.device,
                    dtype=torch.float32 if out_f32 else torch.bfloat16)
    d = dict(geom, H=H, W=W, Ho=Ho, Wo=Wo, stride=stride, pad=pad, relu=int(relu),
             in_f32=int(x.dtype == torch.float32), out_f32=int(out_f32))
    res_ptr = 0
    if residual is not None:
        _check(residual, torch.bfloat16, "residual")
        _, rh, rw, rc = residual.shape
        d.update(has_res=1, res_H=rh, res_W=rw, res_C=rc, res_stride=2 if res_mode == "pad" else 1)
        res_ptr = residual.data_ptr()
    native().conv2d(d, B, x.data_ptr(), w_packed.data_ptr(), bias.data_ptr(), 0, res_ptr,
                    y.data_ptr(), _stream())
    return y


def bottleneck56(x: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor,
                 b2: torch.Tensor, w3: torch.Tensor, b3: torch.Tensor,
                 wd: Optional[torch.Tensor] = None,
                 bd: Optional[torch.Tensor] = None) -> torch.Tensor:
    """One whole ResNet-50 56x56 bottleneck in one kernel (bottleneck_fused.hip).

    x: [B,56,56,256] bf16 (identity shortcut) or [B,56,56,64] with the projection (wd, bd) of
    block 0. Weights packed by ``pack_conv`` (w1 1x1 -> 64, w2 3x3 64 -> 64, w3 / wd 1x1 -> 256).
    Returns relu(conv3(relu(conv2(relu(conv1(x))))) + shortcut), bf16 [B,56,56,256].
    """
    B, H, W, C = x.shape
    down = wd is not None
    if not native().bottleneck56_supported(H, W, C, 64, 256, int(down)):
        raise ValueError(f"bottleneck56: unsupported input {tuple(x.shape)} (down={down})")
    _check(x, torch.bfloat16, "x")
    shapes = {"w1": (w1, (64, C)), "w2": (w2, (64, 576)), "w3": (w3, (256, 64))}
    if down:
        if bd is None:
            raise ValueError("bottleneck56: wd needs bd")
        shapes["wd"] = (wd, (256, 64))
    for name, (t, shp) in shapes.items():
        _check(t, torch.bfloat16, name)
        if tuple(t.shape) != shp:
            raise ValueError(f"bottleneck56: {name} must be {shp}, got {tuple(t.shape)}")
    for name, t, n in (("b1", b1, 64), ("b2", b2, 64), ("b3", b3, 256)) + \
            ((("bd", bd, 256),) if down else ()):
        _check(t, torch.float32, name)
        if t.numel() != n:
            raise ValueError(f"bottleneck56: {name} must have {n} entries")
    y = torch.empty(B, H, W, 256, device=x.device, dtype=torch.bfloat16)
    native().bottleneck56(B, x.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                          b2.data_ptr(), w3.data_ptr(), b3.data_ptr(),
                          wd.data_ptr() if down else 0, bd.data_ptr() if down else 0,
                          y.data_ptr(), C, int(down), _stream())
    return y


def maxpool2d(x: torch.Tensor, k: int, s: int, p: int = 0) -> torch.Tensor:
    _check(x, torch.bfloat16, "x")
    B, H, W, C = x.shape
    Ho = (H + 2 * p - k) // s + 1
    Wo = (W + 2 * p - k) // s + 1
    y = torch.empty(B, Ho, Wo, C, device=x.device, dtype=torch.bfloat16)
    native().maxpool2d(B, H, W, C, k, s, p, Ho, Wo, x.data_ptr(), y.data_ptr(), _stream())
    return y


def avgpool_global(x: torch.Tensor) -> torch.Tensor:
    _check(x, torch.bfloat16, "x")
    B, H, W, C = x.shape
    y = torch.empty(B, C, device=x.device, dtype=torch.bfloat16)
    native().avgpool_global(B, H * W, C, x.data_ptr(), y.data_ptr(), _stream())
    return y


def head(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Global avg pool + dense(fp32 w [N, C]) + softmax. x: [B,H,W,C] bf16 -> [B,N] fp32."""
    _check(x, torch.bfloat16, "x")
    _check(w, torch.float32, "w")
    _check(b, torch.float32, "b")
    B, H, W, C = x.shape
    N = w.shape[0]
    out = torch.empty(B, N, device=x.device, dtype=torch.float32)
    native().head_pool_dense_softmax(B, H * W, C, N, x.data_ptr(), w.data_ptr(), b.data_ptr(),
                                     out.data_ptr(), _stream())
    return out


def softmax(x: torch.Tensor, n: Optional[int] = None) -> torch.Tensor:
    _check(x, torch.float32, "x")
    B, ld = x.shape
    n = ld if n is None else n
    out = torch.empty(B, n, device=x.device, dtype=torch.float32)
    native().softmax_rows(B, n, ld, x.data_ptr(), out.data_ptr(), _stream())
    return out


def batchnorm(x: torch.Tensor, scale: Optional[torch.Tensor], shift: Optional[torch.Tensor],
              relu: bool = False, residual: Optional[torch.Tensor] = None,
              res_mode: str = "identity", out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Inference BatchNorm as a per-channel affine (scale = gamma/sqrt(var+eps),
    shift = beta - mean*scale; None = identity), + optional residual + ReLU. x: [B,H,W,C] bf16
    (C % 8 == 0); scale/shift: fp32 [>= C]. ``res_mode="pad"``: ResNet option-A shortcut
    (residual read at (2h, 2w), zero above its channel count). ``out`` may alias ``x``."""
    _check(x, torch.bfloat16, "x")
    B, H, W, C = x.shape
    if C % 8:
        raise ValueError("batchnorm: channel count must be a multiple of 8")
    sp = hp = 0
    if scale is not None:
        _check(scale, torch.float32, "scale")
        _check(shift, torch.float32, "shift")
        if scale.device != x.device or shift.device != x.device:
            raise ValueError("batchnorm: scale/shift must be on x's device")
        if scale.numel() < C or shift.numel() < C:
            raise ValueError("batchnorm: scale/shift shorter than the channel count")
        sp, hp = scale.data_ptr(), shift.data_ptr()
    rp, rh, rw, rc, rs = 0, 0, 0, 0, 1
    if residual is not None:
        _check(residual, torch.bfloat16, "residual")
        if residual.device != x.device:
            raise ValueError("batchnorm: residual must be on x's device")
        rb, rh, rw, rc = residual.shape
        if res_mode not in ("identity", "pad"):
            raise ValueError(f"batchnorm: unknown res_mode {res_mode!r}")
        rs = 2 if res_mode == "pad" else 1
        if rb != B:
            raise ValueError(f"batchnorm: residual batch {rb} != {B}")
        if res_mode == "identity" and (rh, rw, rc) != (H, W, C):
            raise ValueError(f"batchnorm: identity residual {tuple(residual.shape)} != "
                             f"{tuple(x.shape)}")
        if res_mode == "pad" and (rh < 2 * (H - 1) + 1 or rw < 2 * (W - 1) + 1 or rc > C):
            raise ValueError(f"batchnorm: pad residual {tuple(residual.shape)} does not cover "
                             f"{tuple(x.shape)} at stride 2")
        rp = residual.data_ptr()
    if out is None:
        y = torch.empty_like(x)
    else:
        _check(out, torch.bfloat16, "out")
        if out.shape != x.shape or out.device != x.device:
            raise ValueError(f"batchnorm: out {tuple(out.shape)} on {out.device} must match x "
                             f"{tuple(x.shape)} on {x.device}")
        y = out
    native().bn_act(B, H * W, W, C, x.data_ptr(), sp, hp, rp, rh, rw, rc, rs, int(relu),
                    y.data_ptr(), _stream())
    return y


def relu(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Standalone ReLU over a bf16 NHWC tensor (the conv epilogue fuses it on the fast path)."""
    return batchnorm(x, None, None, relu=True, out=out)


def cast_bf16(x: torch.Tensor, scale: float = 1.0, shift: float = 0.0) -> torch.Tensor:
    _check(x, torch.float32, "x")
    y = torch.empty(x.shape, device=x.device, dtype=torch.bfloat16)
    native().cast_f32_bf16(x.numel(), scale, shift, x.data_ptr(), y.data_ptr(), _stream())
    return y


# ---- fp8 (OCP e4m3fn) path: tensors of e4m3 codes are uint8 --------------------------------


def pack_conv_fp8(w_oihw: torch.Tensor, bias: torch.Tensor, cin_stored: Optional[int] = None,
                  device=None):
    """Pack an fp32 conv weight as e4m3 codes with per-output-channel scales.

    Returns (w codes uint8 [Npad, Kpad], bias fp32 [Npad], wscale fp32 [Npad], geometry dict).
    """
    from gale.models.quant import quantize_rows_e4m3

    cout, cin, kh, kw = w_oihw.shape
    cin_s = cin if cin_stored is None else cin_stored
    cout_s = round_up(cout, 4)
    K = kh * kw * cin_s
    Kpad = round_up(K, 32)
    Npad = round_up(cout_s, conv_n_tiles(cout_s) * 16)
    q, s = quantize_rows_e4m3(pack_conv_weight(w_oihw.float().cpu(), cin_s, Npad, Kpad))
    bp = torch.zeros(Npad)
    bp[:cout] = bias.float().cpu()
    dev = device if device is not None else torch.device("cuda")
    return q.to(dev), bp.to(dev), s.to(dev), dict(Cin=cin_s, Cout=cout_s, KH=kh, KW=kw, K=K,
                                                   Kpad=Kpad, Npad=Npad)


def conv2d_fp8(x: torch.Tensor, w_codes: torch.Tensor, bias: torch.Tensor, wscale: torch.Tensor,
               geom: dict, in_scale: float, out_scale: float = 1.0, stride: int = 1, pad: int = 0,
               relu: bool = False, residual: Optional[torch.Tensor] = None,
               res_scale: float = 1.0, res_mode: str = "identity",
               out_f32: bool = False) -> torch.Tensor:
    """NHWC conv on fp8 MFMA. x: e4m3 codes (uint8, value = code * in_scale) or fp32 (quantised
    with step in_scale while loaded). Returns e4m3 codes at out_scale, or fp32 (out_f32)."""
    B, H, W, C = x.shape
    if C != geom["Cin"]:
        raise ValueError(f"x has {C} channels, packed weight expects {geom['Cin']}")
    _check(w_codes, torch.uint8, "w_codes")
    _check(bias, torch.float32, "bias")
    _check(wscale, torch.float32, "wscale")
    if x.dtype not in (torch.uint8, torch.float32):
        raise TypeError("x must be e4m3 codes (uint8) or fp32")
    _check(x, x.dtype, "x")
    kh, kw = geom["KH"], geom["KW"]
    Ho = (H + 2 * pad - kh) // stride + 1
    Wo = (W + 2 * pad - kw) // stride + 1
    y = torch.empty(B, Ho, Wo, geom["Cout"], device=x.device,
                    dtype=torch.float32 if out_f32 else torch.uint8)
    d = dict(geom, H=H, W=W, Ho=Ho, Wo=Wo, stride=stride, pad=pad, relu=int(relu),
             in_f32=int(x.dtype == torch.float32), out_f32=int(out_f32), fp8=1,
             in_scale=float(in_scale), out_scale=float(out_scale), res_scale=float(res_scale))
    res_ptr = 0
    if residual is not None:
        _check(residual, torch.uint8, "residual")
        _, rh, rw, rc = residual.shape
        d.update(has_res=1, res_H=rh, res_W=rw, res_C=rc, res_stride=2 if res_mode == "pad" else 1)
        res_ptr = residual.data_ptr()
    native().conv2d(d, B, x.data_ptr(), w_codes.data_ptr(), bias.data_ptr(), wscale.data_ptr(),
                    res_ptr, y.data_ptr(), _stream())
    return y


def maxpool2d_fp8(x: torch.Tensor, k: int, s: int, p: int = 0) -> torch.Tensor:
    _check(x, torch.uint8, "x")
    B, H, W, C = x.shape
    Ho = (H + 2 * p - k) // s + 1
    Wo = (W + 2 * p - k) // s + 1
    y = torch.empty(B, Ho, Wo, C, device=x.device, dtype=torch.uint8)
    native().maxpool2d(B, H, W, C, k, s, p, Ho, Wo, x.data_ptr(), y.data_ptr(), _stream(), 1)
    return y


def avgpool_global_fp8(x: torch.Tensor) -> torch.Tensor:
    _check(x, torch.uint8, "x")
    B, H, W, C = x.shape
    y = torch.empty(B, C, device=x.device, dtype=torch.uint8)
    native().avgpool_global(B, H * W, C, x.data_ptr(), y.data_ptr(), _stream(), 1)
    return y


def head_fp8(x: torch.Tensor, in_scale: float, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    _check(x, torch.uint8, "x")
    _check(w, torch.float32, "w")
    _check(b, torch.float32, "b")
    B, H, W, C = x.shape
    N = w.shape[0]
    out = torch.empty(B, N, device=x.device, dtype=torch.float32)
    native().head_pool_dense_softmax(B, H * W, C, N, x.data_ptr(), w.data_ptr(), b.data_ptr(),
                                     out.data_ptr(), _stream(), 1, float(in_scale))
    return out
