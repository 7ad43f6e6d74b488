"""Host-side conv dispatch rules (no GPU needed): which layer shapes take the LDS halo-patch 3x3
kernel (conv_patch.hip) under each set_conv_patch mode, and which stay on the im2col GEMM."""

import torch

from gale import ops
from gale._native import native


def _desc(H, Cin, Cout, k=3, stride=1, pad=1, res=False):
    w = torch.zeros(Cout, Cin, k, k)
    _, _, geom = ops.pack_conv(w, torch.zeros(Cout), device="cpu")
    Ho = (H + 2 * pad - k) // stride + 1
    d = dict(geom, H=H, W=H, Ho=Ho, Wo=Ho, stride=stride, pad=pad, relu=1, in_f32=0, out_f32=0)
    if res:
        d.update(has_res=1, res_H=Ho, res_W=Ho, res_C=geom["Cout"], res_stride=1)
    return d


def test_conv_patch_dispatch_rules():
    C = native()
    try:
        C.set_conv_patch(1)  # default: 128-channel tiles only
        assert C.conv_patch_supported(_desc(28, 128, 128), 256, False)
        assert C.conv_patch_supported(_desc(14, 256, 256), 256, False)
        assert C.conv_patch_supported(_desc(7, 512, 512), 3, False)      # two images per tile
        assert C.conv_patch_supported(_desc(28, 128, 128, res=True), 4, True)
        assert not C.conv_patch_supported(_desc(56, 64, 64), 256, False)  # 64-channel tile
        assert not C.conv_patch_supported(_desc(28, 128, 128, stride=2), 256, False)
        assert not C.conv_patch_supported(_desc(28, 128, 128, k=1, pad=0), 256, False)
        assert not C.conv_patch_supported(_desc(28, 96, 128), 256, False)  # Cin % 64
        C.set_conv_patch(2)  # + 64-channel tiles
        assert C.conv_patch_supported(_desc(56, 64, 64), 256, False)
        C.set_conv_patch(0)
        assert not C.conv_patch_supported(_desc(28, 128, 128), 256, False)
        C.set_conv_patch(1)
        C.set_conv_path(1)  # "never the GEMM paths" covers the patch kernel too
        assert not C.conv_patch_supported(_desc(28, 128, 128), 256, False)
    finally:
        C.set_conv_path(0)
        C.set_conv_patch(1)
