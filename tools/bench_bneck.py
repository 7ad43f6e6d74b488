"""Time the fused 56x56 bottleneck kernel alone (bottleneck_fused.hip) at ResNet-50 batch 256,
identity and projection forms, against the layered kernels it replaces. One JSON line per form."""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--layered", action="store_true", help="also time the layered kernels")
    a = ap.parse_args()
    from gale import ops

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    for down in (False, True):
        cin = 64 if down else 256
        x = torch.randn(a.batch, 56, 56, cin, generator=g).to(dev, torch.bfloat16)

        def pk(cout, ci, k):
            w = torch.randn(cout, ci, k, k, generator=g) * (2.0 / (k * k * ci)) ** 0.5
            return ops.pack_conv(w, torch.randn(cout, generator=g) * 0.1, device=dev)
        (w1, b1, g1), (w2, b2, g2), (w3, b3, g3) = pk(64, cin, 1), pk(64, 64, 3), pk(256, 64, 1)
        wd = bd = gd = None
        if down:
            wd, bd, gd = pk(256, cin, 1)

        def fused():
            return ops.bottleneck56(x, w1, b1, w2, b2, w3, b3, wd, bd)

        def layered():
            h = ops.conv2d(x, w1, b1, g1, relu=True)
            h = ops.conv2d(h, w2, b2, g2, pad=1, relu=True)
            sc = ops.conv2d(x, wd, bd, gd) if down else x
            return ops.conv2d(h, w3, b3, g3, relu=True, residual=sc)

        for name, fn in [("fused", fused)] + ([("layered", layered)] if a.layered else []):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            print(json.dumps(dict(form="down" if down else "identity", impl=name, batch=a.batch,
                                  us=round(us, 1))),
                  flush=True)


if __name__ == "__main__":
    main()
