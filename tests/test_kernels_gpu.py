"""Numerics of the hand-written gfx950 kernels against plain PyTorch fp32 references.

Operands are asymmetric random data (cdna_hip_programming.md §3: a symmetric operand hides a
transposed C-write). Tolerances are bf16-level: inputs/weights are rounded to bf16 and the
reference uses the same rounded values, so the remaining error is fp32-accumulation order plus
the bf16 rounding of the output.
"""

import pytest
import torch
import torch.nn.functional as F

from gale import ops

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ref_conv(x_nhwc, w, b, stride, pad, relu, res=None, res_mode="identity"):
    x = x_nhwc.float().permute(0, 3, 1, 2)
    y = F.conv2d(x, w.float(), b.float(), stride=stride, padding=pad)
    if res is not None:
        r = res.float().permute(0, 3, 1, 2)
        if res_mode == "pad":
            r = r[:, :, ::2, ::2]
            r = F.pad(r, (0, 0, 0, 0, 0, y.shape[1] - r.shape[1]))
        y = y + r
    if relu:
        y = F.relu(y)
    return y.permute(0, 2, 3, 1)


CONV_CASES = [
    # B, H, W, Cin, Cout, k, stride, pad, in_f32
    (3, 32, 32, 3, 16, 3, 1, 1, True),      # ResNet-20 stem (gather, fp32 input)
    (2, 28, 28, 1, 8, 5, 1, 2, True),       # LeNet conv1
    (4, 32, 32, 16, 16, 3, 1, 1, False),    # ResNet-20 stage 1
    (4, 32, 32, 16, 32, 3, 2, 1, False),    # stage 2 downsample
    (3, 16, 16, 32, 32, 3, 1, 1, False),
    (5, 8, 8, 64, 64, 3, 1, 1, False),      # stage 3
    (2, 5, 5, 16, 120, 5, 1, 0, False),     # LeNet fc1 as a 5x5 valid conv
    (3, 14, 14, 64, 256, 1, 1, 0, False),   # ResNet-50 1x1 expand (n-blocks > 1)
    (2, 14, 14, 256, 128, 1, 2, 0, False),  # 1x1 stride-2 projection
    (2, 7, 7, 512, 512, 3, 1, 1, False),    # K = 4608: K-chunked (non weight-stationary)
    (1, 56, 56, 64, 64, 3, 1, 1, False),
]


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("relu", [False, True])
def test_conv2d_matches_torch(case, relu):
    B, H, W, Cin, Cout, k, s, p, in_f32 = case
    g = torch.Generator().manual_seed(1234 + Cin * 7 + Cout)
    x = torch.randn(B, H, W, Cin, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.1
    xq = x if in_f32 else x.to(torch.bfloat16)
    wq = w.to(torch.bfloat16).float()
    wp, bp, geom = ops.pack_conv(w, b)
    y = ops.conv2d(xq.to(DEV), wp, bp, geom, stride=s, pad=p, relu=relu)
    ref = _ref_conv(xq.to(torch.bfloat16).float(), wq, b, s, p, relu)
    torch.cuda.synchronize()
    got = y.float().cpu()[..., :Cout]
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err <= 2e-2 * scale + 1e-2, f"max err {err} (scale {scale})"


@pytest.mark.parametrize("mode", ["identity", "pad"])
def test_conv2d_residual(mode):
    g = torch.Generator().manual_seed(7)
    B, H, Cin, Cout = 3, 16, 16 if mode == "pad" else 32, 32
    s = 2 if mode == "pad" else 1
    Hin = H * s
    x = torch.randn(B, Hin, Hin, Cin, generator=g).to(torch.bfloat16)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / (Cin * 9) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.1
    res_c = Cin if mode == "pad" else Cout
    res = torch.randn(B, Hin if mode == "pad" else H, Hin if mode == "pad" else H, res_c,
                      generator=g).to(torch.bfloat16)
    wp, bp, geom = ops.pack_conv(w, b)
    y = ops.conv2d(x.to(DEV), wp, bp, geom, stride=s, pad=1, relu=True, residual=res.to(DEV),
                   res_mode=mode)
    ref = _ref_conv(x.float(), w.to(torch.bfloat16).float(), b, s, 1, True, res=res, res_mode=mode)
    err = (y.float().cpu() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-2


def test_conv2d_identity_weight_asymmetric():
    """A = I check: a 1x1 conv with identity weights must reproduce an asymmetric input exactly."""
    B, H, C = 2, 8, 64
    x = (torch.arange(B * H * H * C, dtype=torch.float32).reshape(B, H, H, C) % 97) / 8.0
    x = x.to(torch.bfloat16)
    w = torch.eye(C).reshape(C, C, 1, 1)
    wp, bp, geom = ops.pack_conv(w, torch.zeros(C))
    y = ops.conv2d(x.to(DEV), wp, bp, geom)
    assert torch.equal(y.cpu(), x)


def test_conv2d_fc_out_f32():
    g = torch.Generator().manual_seed(3)
    B, K, N = 9, 2048, 1000
    x = torch.randn(B, 1, 1, K, generator=g).to(torch.bfloat16)
    w = torch.randn(N, K, 1, 1, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g)
    wp, bp, geom = ops.pack_conv(w, b)
    y = ops.conv2d(x.to(DEV), wp, bp, geom, out_f32=True)
    assert y.dtype == torch.float32
    ref = x.float().reshape(B, K) @ w.reshape(N, K).to(torch.bfloat16).float().t() + b
    err = (y.cpu().reshape(B, N) - ref).abs().max().item()
    assert err < 1e-2 * ref.abs().max().item() + 1e-3


@pytest.mark.parametrize("k,s,p", [(2, 2, 0), (3, 2, 1)])
def test_maxpool(k, s, p):
    x = torch.randn(3, 28, 28, 16).to(torch.bfloat16)
    y = ops.maxpool2d(x.to(DEV), k, s, p).cpu()
    ref = F.max_pool2d(x.float().permute(0, 3, 1, 2), k, s, p).permute(0, 2, 3, 1)
    assert torch.equal(y.float(), ref)


def test_avgpool_and_head_and_softmax():
    g = torch.Generator().manual_seed(5)
    x = torch.randn(6, 8, 8, 64, generator=g).to(torch.bfloat16)
    pooled = ops.avgpool_global(x.to(DEV)).float().cpu()
    ref_pool = x.float().mean(dim=(1, 2))
    assert (pooled - ref_pool).abs().max().item() < 1e-2
    w = torch.randn(10, 64, generator=g) * 0.3
    b = torch.randn(10, generator=g) * 0.1
    probs = ops.head(x.to(DEV), w.to(DEV), b.to(DEV)).cpu()
    ref = torch.softmax(ref_pool @ w.t() + b, dim=1)
    assert (probs - ref).abs().max().item() < 1e-4
    assert torch.allclose(probs.sum(1), torch.ones(6), atol=1e-5)
    logits = torch.randn(5, 1000, generator=g) * 3
    sm = ops.softmax(logits.to(DEV)).cpu()
    assert (sm - torch.softmax(logits, 1)).abs().max().item() < 1e-6


def test_cast():
    x = torch.randn(1024)
    y = ops.cast_bf16(x.to(DEV), 2.0, 0.5).cpu()
    assert torch.equal(y, (x * 2.0 + 0.5).to(torch.bfloat16))


def test_no_cpu_fallback():
    w, b, geom = ops.pack_conv(torch.randn(16, 16, 3, 3), torch.zeros(16))
    with pytest.raises(RuntimeError):
        ops.conv2d(torch.randn(1, 8, 8, 16).to(torch.bfloat16), w, b, geom)


# ---- fp8 (OCP e4m3fn) kernels -------------------------------------------------------------

def _e4m3(t):
    from gale.models.quant import e4m3_codes
    return e4m3_codes(t)


def _from_e4m3(codes):
    return codes.view(torch.float8_e4m3fn).float()


def test_conv2d_fp8_exact_small_integers():
    """Exact check of the fp8 MFMA operand layout: small integers are exact in e4m3 and every
    partial sum is exact in fp32, so the result must match bit for bit (asymmetric operands)."""
    g = torch.Generator().manual_seed(21)
    B, H, Cin, Cout = 2, 8, 32, 48
    xv = torch.randint(-3, 4, (B, H, H, Cin), generator=g).float()
    w = torch.randint(-3, 4, (Cout, Cin, 3, 3), generator=g).float() * 0.25
    w[:, 0, 0, 0] = 0.875  # every row max is 448/512: power-of-two scale 1/512, codes exact
    from gale import ops
    wq, bq, ws, geom = ops.pack_conv_fp8(w, torch.zeros(Cout))
    y = ops.conv2d_fp8(_e4m3(xv).to(DEV), wq, bq, ws, geom, in_scale=1.0, stride=1, pad=1,
                       out_scale=4.0)
    ref = _ref_conv(xv, w, torch.zeros(Cout), 1, 1, False)
    # outputs are multiples of 1/4 (exact fp32 sums and scale products): both round v/4 to e4m3
    got = _from_e4m3(y.cpu())
    from gale.models.quant import e4m3_round
    assert torch.equal(got[..., :Cout], e4m3_round(ref / 4.0))


@pytest.mark.parametrize("case", [c for c in CONV_CASES if c[3] <= 256])
def test_conv2d_fp8_matches_emulation(case):
    B, H, W, Cin, Cout, k, s, p, in_f32 = case
    g = torch.Generator().manual_seed(99 + Cin + Cout)
    x = torch.randn(B, H, W, Cin, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.1
    from gale import ops
    from gale.models.quant import e4m3_round, fake_quant_weight
    in_scale = float(x.abs().max()) / 448
    xq = e4m3_round(x / in_scale) * in_scale  # the values the kernel consumes
    ref = _ref_conv(xq, fake_quant_weight(w), b, s, p, True)
    out_scale = float(ref.abs().max()) / 448
    wq, bq, ws, geom = ops.pack_conv_fp8(w, b)
    xin = x.to(DEV) if in_f32 else _e4m3(x / in_scale).to(DEV)
    y = ops.conv2d_fp8(xin, wq, bq, ws, geom, in_scale=in_scale, out_scale=out_scale, stride=s,
                       pad=p, relu=True)
    got = _from_e4m3(y.cpu())[..., :Cout] * out_scale
    # same quantised operands; remaining differences: fp32 summation order + one e4m3 rounding
    err = (got - e4m3_round(ref / out_scale) * out_scale).abs()
    assert err.max().item() <= 0.0625 * float(ref.abs().max()) + 1e-6
    assert err.mean().item() <= 1e-3 * float(ref.abs().max()) + 1e-6


def test_conv2d_fp8_residual_and_out_f32():
    g = torch.Generator().manual_seed(8)
    from gale import ops
    from gale.models.quant import e4m3_round, fake_quant_weight
    B, Hin, Cin, Cout = 2, 16, 16, 32
    x = torch.rand(B, Hin, Hin, Cin, generator=g)
    res = torch.rand(B, Hin, Hin, Cin, generator=g) * 2
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / (Cin * 9) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.1
    sx, sr = 1 / 448, 2 / 448
    wq, bq, ws, geom = ops.pack_conv_fp8(w, b)
    y = ops.conv2d_fp8(_e4m3(x / sx).to(DEV), wq, bq, ws, geom, in_scale=sx, out_scale=4 / 448,
                       stride=2, pad=1, relu=True, residual=_e4m3(res / sr).to(DEV),
                       res_scale=sr, res_mode="pad")
    ref = _ref_conv(e4m3_round(x / sx) * sx, fake_quant_weight(w), b, 2, 1, True,
                    res=e4m3_round(res / sr) * sr, res_mode="pad")
    got = _from_e4m3(y.cpu()) * (4 / 448)
    assert (got - ref).abs().max().item() < 0.07 * float(ref.abs().max())
    # fc layer with fp32 logits out
    K, N = 512, 100
    xf = torch.rand(5, 1, 1, K, generator=g)
    wf = torch.randn(N, K, 1, 1, generator=g) / K ** 0.5
    wq, bq, ws, geom = ops.pack_conv_fp8(wf, torch.zeros(N))
    yl = ops.conv2d_fp8(_e4m3(xf * 448).to(DEV), wq, bq, ws, geom, in_scale=1 / 448, out_f32=True)
    refl = (e4m3_round(xf * 448) / 448).reshape(5, K) @ fake_quant_weight(wf).reshape(N, K).t()
    assert (yl.cpu().reshape(5, -1)[:, :N] - refl).abs().max().item() < 1e-4


def test_pool_and_head_fp8():
    g = torch.Generator().manual_seed(4)
    from gale import ops
    x = torch.randn(3, 12, 12, 16, generator=g) * 50
    codes = _e4m3(x)
    xv = _from_e4m3(codes)
    y = ops.maxpool2d_fp8(codes.to(DEV), 3, 2, 1).cpu()
    ref = F.max_pool2d(xv.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.equal(_from_e4m3(y), ref)
    pooled = _from_e4m3(ops.avgpool_global_fp8(codes.to(DEV)).cpu())
    from gale.models.quant import e4m3_round
    assert torch.allclose(pooled, e4m3_round(xv.mean(dim=(1, 2))), rtol=0.07, atol=0.02)
    w = torch.randn(10, 16, generator=g) * 0.01
    b = torch.randn(10, generator=g) * 0.1
    probs = ops.head_fp8(codes.to(DEV), 0.5, w.to(DEV), b.to(DEV)).cpu()
    refp = torch.softmax((xv * 0.5).mean(dim=(1, 2)) @ w.t() + b, dim=1)
    assert (probs - refp).abs().max().item() < 1e-4


GEMM_CASES = [
    # B, H, W, Cin, Cout, k, stride, pad, residual
    (2, 14, 14, 64, 64, 3, 1, 1, False),      # ResNet-50 stage 1 3x3 (BN = 64), M % 128 != 0
    (3, 9, 11, 64, 128, 3, 2, 1, True),       # strided 3x3, odd sizes, BN = 128, residual
    (2, 14, 14, 256, 128, 1, 2, 0, False),    # 1x1 stride-2 projection
    (4, 7, 7, 128, 512, 1, 1, 0, True),       # 1x1 expand + residual
    (1, 7, 7, 512, 512, 3, 1, 1, False),      # K = 4608 (72 k-steps)
]


@pytest.mark.parametrize("case", GEMM_CASES)
def test_conv2d_gemm_path_matches_torch(case):
    """The LDS-pipelined GEMM conv (conv_gemm.hip), forced on small shapes, vs fp32 torch."""
    from gale._native import native

    B, H, W, Cin, Cout, k, s, p, with_res = case
    g = torch.Generator().manual_seed(99 + Cin + Cout + k)
    x = torch.randn(B, H, W, Cin, generator=g).to(torch.bfloat16)
    w = torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.1
    wp, bp, geom = ops.pack_conv(w, b)
    Ho = (H + 2 * p - k) // s + 1
    Wo = (W + 2 * p - k) // s + 1
    res = torch.randn(B, Ho, Wo, Cout, generator=g).to(torch.bfloat16) if with_res else None
    C = native()
    try:
        C.set_conv_path(2)
        y = ops.conv2d(x.to(DEV), wp, bp, geom, stride=s, pad=p, relu=True,
                       residual=None if res is None else res.to(DEV))
        C.set_conv_path(1)
        y_old = ops.conv2d(x.to(DEV), wp, bp, geom, stride=s, pad=p, relu=True,
                           residual=None if res is None else res.to(DEV))
    finally:
        C.set_conv_path(0)
    ref = _ref_conv(x.float(), w.to(torch.bfloat16).float(), b, s, p, True, res=res)
    got = y.float().cpu()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err <= 2e-2 * scale + 1e-2, f"max err {err} (scale {scale})"
    # both paths accumulate in fp32 and round once to bf16: they agree to one bf16 ulp
    assert (y.float() - y_old.float()).abs().max().item() <= 1e-2 * scale + 1e-2


def test_conv2d_gemm_identity_asymmetric():
    """A = I check on the GEMM path: 1x1 identity weights reproduce an asymmetric input exactly
    (catches a transposed C-write or a wrong LDS swizzle)."""
    from gale._native import native

    B, H, C = 2, 12, 128
    x = (torch.arange(B * H * H * C, dtype=torch.float32).reshape(B, H, H, C) % 251) / 16.0
    x = x.to(torch.bfloat16)
    w = torch.eye(C).reshape(C, C, 1, 1)
    wp, bp, geom = ops.pack_conv(w, torch.zeros(C))
    try:
        native().set_conv_path(2)
        y = ops.conv2d(x.to(DEV), wp, bp, geom)
    finally:
        native().set_conv_path(0)
    assert torch.equal(y.cpu(), x)


def test_stem_pack_layout():
    """stem_pack: fp32 NHWC (C=3) -> bf16 [H][Wp][4] with lp zero columns on the left, zero
    right padding and a zero 4th channel (the packed-stem input, conv_gemm.hip)."""
    from gale._native import native

    B, H, W, C, lp = 2, 5, 7, 3, 3
    Wp = W + 2 * lp + 1
    x = torch.randn(B, H, W, C, generator=torch.Generator().manual_seed(4))
    y = torch.full((B, H, Wp, 4), 7.0, dtype=torch.bfloat16, device=DEV)
    xd = x.to(DEV)
    native().stem_pack(B, H, W, C, Wp, lp, xd.data_ptr(), y.data_ptr(),
                       torch.cuda.current_stream().cuda_stream)
    ref = torch.zeros(B, H, Wp, 4)
    ref[:, :, lp:lp + W, :C] = x
    assert torch.equal(y.cpu(), ref.to(torch.bfloat16))


@pytest.mark.parametrize("mode", ["none", "identity", "pad"])
def test_batchnorm_residual_relu(mode):
    """Standalone inference BatchNorm (+ residual + ReLU) vs fp32, incl. the option-A shortcut."""
    g = torch.Generator().manual_seed(8)
    B, H, W, C = 3, 8, 10, 32
    x = (torch.randn(B, H, W, C, generator=g) * 2).bfloat16()
    scale = torch.rand(C, generator=g) + 0.5
    shift = torch.randn(C, generator=g)
    ref = x.float() * scale + shift
    res = None
    if mode == "identity":
        res = torch.randn(B, H, W, C, generator=g).bfloat16()
        ref = ref + res.float()
    elif mode == "pad":
        res = torch.randn(B, 2 * H, 2 * W, 16, generator=g).bfloat16()
        ref[..., :16] += res.float()[:, ::2, ::2, :]
    ref = ref.clamp(min=0)
    y = ops.batchnorm(x.to(DEV), scale.to(DEV), shift.to(DEV), relu=True,
                      residual=None if res is None else res.to(DEV),
                      res_mode="pad" if mode == "pad" else "identity").float().cpu()
    assert torch.all((y - ref).abs() <= ref.abs() * 8e-3 + 1e-3)


def test_relu_standalone_in_place():
    x = torch.randn(2, 5, 7, 24, generator=torch.Generator().manual_seed(2)).bfloat16().to(DEV)
    want = x.clamp(min=0).cpu()
    y = ops.relu(x, out=x)
    assert y.data_ptr() == x.data_ptr() and torch.equal(x.cpu(), want)


def test_batchnorm_rejects_mismatched_operands():
    """Shape/device/dtype errors are Python errors, never out-of-bounds device accesses."""
    x = torch.randn(2, 4, 4, 16).bfloat16().to(DEV)
    sc, sh = torch.ones(16, device=DEV), torch.zeros(16, device=DEV)
    with pytest.raises(ValueError):  # short out
        ops.batchnorm(x, sc, sh, out=torch.empty(1, 4, 4, 16, dtype=torch.bfloat16, device=DEV))
    with pytest.raises(ValueError):  # residual batch
        ops.batchnorm(x, sc, sh, residual=torch.zeros(1, 4, 4, 16, dtype=torch.bfloat16,
                                                      device=DEV))
    with pytest.raises(ValueError):  # identity residual of another shape
        ops.batchnorm(x, sc, sh, residual=torch.zeros(2, 4, 4, 8, dtype=torch.bfloat16,
                                                      device=DEV))
    with pytest.raises(RuntimeError):  # scale on the host (no CPU fallback)
        ops.batchnorm(x, torch.ones(16), torch.zeros(16))
    with pytest.raises(TypeError):  # out dtype
        ops.batchnorm(x, sc, sh, out=torch.empty(2, 4, 4, 16, device=DEV))


@pytest.mark.parametrize("B,H,W,Cin,Cout,k,stride,pad,res", [
    (3, 32, 32, 3, 16, 3, 1, 1, None),       # network-input gather (Cin 3)
    (4, 16, 16, 16, 32, 3, 2, 1, "pad"),     # stride 2 + option-A shortcut
    (2, 8, 8, 64, 72, 3, 1, 1, "identity"),  # Cout not a multiple of the 64-channel tile
    (5, 7, 7, 40, 24, 1, 1, 0, None),        # 1x1
])
def test_conv_f32_matches_fp32(B, H, W, Cin, Cout, k, stride, pad, res):
    """The fp32-MFMA conv (conv_f32.hip) against an fp32 conv: summation-order-level error."""
    from gale._native import native
    from gale.models.graph import pack_conv_weight, round_up

    g = torch.Generator().manual_seed(B * 100 + Cout)
    x = torch.randn(B, H, W, Cin, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) / (k * k * Cin) ** 0.5
    b = torch.randn(Cout, generator=g)
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    r = None
    if res == "identity":
        r = torch.randn(B, Ho, Wo, Cout, generator=g)
    elif res == "pad":
        r = torch.randn(B, H, W, Cin, generator=g)
    K = k * k * Cin
    Kpad = round_up(K, 16)
    wp = pack_conv_weight(w, Cin, Cout, Kpad).to(DEV)
    y = torch.empty(B, Ho, Wo, Cout, device=DEV)
    d = dict(H=H, W=W, Cin=Cin, Ho=Ho, Wo=Wo, Cout=Cout, KH=k, KW=k, stride=stride, pad=pad, K=K,
             Kpad=Kpad, Npad=Cout, relu=1, f32=1)
    rd = 0
    if r is not None:
        rd_t = r.to(DEV)
        d.update(has_res=1, res_H=r.shape[1], res_W=r.shape[2], res_C=r.shape[3],
                 res_stride=2 if res == "pad" else 1)
        rd = rd_t.data_ptr()
    xd, bd = x.to(DEV), b.to(DEV)
    native().conv2d(d, B, xd.data_ptr(), wp.data_ptr(), bd.data_ptr(), 0, rd, y.data_ptr(),
                    torch.cuda.current_stream().cuda_stream)
    ref = _ref_conv(x, w, b, stride, pad, True, r, res or "identity")
    got = y.cpu()
    scale = ref.abs().max().item()
    assert (got - ref).abs().max().item() < 2e-5 * max(scale, 1.0)


PATCH_CASES = [  # B, H, W, Cin, Cout, with_res: the ResNet-50 3x3 stride-1 shapes (+ residual)
    (2, 56, 56, 64, 64, False),     # 2 rows x 56 per tile, BN = 64, 240-row patch
    (3, 28, 28, 128, 128, True),    # 4 rows x 28, BN = 128
    (2, 14, 14, 256, 256, False),   # 7 rows x 14 (98 of 128 MFMA rows), two channel tiles
    (1, 14, 14, 128, 64, True),     # BN = 64 at 14 x 14
    (3, 7, 7, 512, 512, True),      # two whole 7 x 7 images per tile, a partial last tile
]


def _patch_desc(geom, B, H, W, has_res):
    d = dict(geom, H=H, W=W, Ho=H, Wo=W, stride=1, pad=1, relu=1, in_f32=0, out_f32=0)
    if has_res:
        d.update(has_res=1, res_H=H, res_W=W, res_C=geom["Cout"], res_stride=1)
    return d


@pytest.mark.parametrize("case", PATCH_CASES)
def test_conv2d_patch_path_matches_torch(case):
    """conv_patch.hip (3x3 stride 1 from an LDS-resident halo patch) vs fp32 torch and vs the
    im2col GEMM path on the same inputs."""
    from gale._native import native

    B, H, W, Cin, Cout, with_res = case
    g = torch.Generator().manual_seed(7 + Cin + Cout + H)
    x = torch.randn(B, H, W, Cin, generator=g).to(torch.bfloat16)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / (Cin * 9) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.1
    wp, bp, geom = ops.pack_conv(w, b)
    res = torch.randn(B, H, W, Cout, generator=g).to(torch.bfloat16) if with_res else None
    C = native()
    try:
        C.set_conv_patch(2)  # (2: the 64-channel tiles too)
        assert C.conv_patch_supported(_patch_desc(geom, B, H, W, with_res), B, with_res)
        y = ops.conv2d(x.to(DEV), wp, bp, geom, stride=1, pad=1, relu=True,
                       residual=None if res is None else res.to(DEV))
        C.set_conv_patch(0)
        y_gemm = ops.conv2d(x.to(DEV), wp, bp, geom, stride=1, pad=1, relu=True,
                            residual=None if res is None else res.to(DEV))
    finally:
        C.set_conv_patch(1)
    ref = _ref_conv(x.float(), w.to(torch.bfloat16).float(), b, 1, 1, True, res=res)
    got = y.float().cpu()
    scale = ref.abs().max().item() + 1e-6
    err = (got - ref).abs().max().item()
    assert err <= 2e-2 * scale + 1e-2, f"max err {err} (scale {scale})"
    assert (y.float() - y_gemm.float()).abs().max().item() <= 1e-2 * scale + 1e-2


@pytest.mark.parametrize("H,C,tap", [(56, 64, 4), (28, 128, 0), (14, 256, 8), (28, 128, 5),
                                     (7, 128, 0), (7, 128, 8)])
def test_conv2d_patch_single_tap_shift_is_exact(H, C, tap):
    """One identity tap (kh, kw) and zeros elsewhere: y[n, i, j] = x[n, i + kh - 1, j + kw - 1]
    (zero outside the image), bit exact - pins the patch-row mapping, the halo and the zero
    padding of every tap position on an asymmetric input."""
    from gale._native import native

    B = 2
    x = (torch.arange(B * H * H * C, dtype=torch.float32).reshape(B, H, H, C) % 251) / 16.0
    x = x.to(torch.bfloat16)
    kh, kw = divmod(tap, 3)
    w = torch.zeros(C, C, 3, 3)
    w[:, :, kh, kw] = torch.eye(C)
    wp, bp, geom = ops.pack_conv(w, torch.zeros(C))
    try:
        native().set_conv_patch(2)
        assert native().conv_patch_supported(_patch_desc(geom, B, H, H, False), B, False)
        y = ops.conv2d(x.to(DEV), wp, bp, geom, stride=1, pad=1).cpu()
    finally:
        native().set_conv_patch(1)
    xp = torch.nn.functional.pad(x.float(), (0, 0, 1, 1, 1, 1))
    want = xp[:, kh:kh + H, kw:kw + H, :].to(torch.bfloat16)
    assert torch.equal(y, want)
