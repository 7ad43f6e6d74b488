"""Time single ResNet-50 body convolutions (batch 256, bf16) on the conv_gemm path: the 3x3/1
layers of stages 2-4 and a 1x1 expansion with its residual. One JSON line per shape."""
import argparse
import json
import os
import sys

import torch

sys.path.append(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gale import ops

SHAPES = {
    "l2.conv2 3x3 28x28 128": dict(H=28, cin=128, cout=128, k=3),
    "l3.conv2 3x3 14x14 256": dict(H=14, cin=256, cout=256, k=3),
    "l4.conv2 3x3 7x7 512": dict(H=7, cin=512, cout=512, k=3),
    "l2.conv3 1x1 28x28 128->512 +res": dict(H=28, cin=128, cout=512, k=1, res=True),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    for name, s in SHAPES.items():
        w = torch.randn(s["cout"], s["cin"], s["k"], s["k"], generator=g) * 0.05
        b = torch.randn(s["cout"], generator=g) * 0.1
        wp, bp, geom = ops.pack_conv(w, b, device=dev)
        x = torch.randn(a.batch, s["H"], s["H"], s["cin"], device=dev).to(torch.bfloat16)
        res = torch.randn(a.batch, s["H"], s["H"], s["cout"], device=dev).to(torch.bfloat16) \
            if s.get("res") else None
        pad = s["k"] // 2

        def run():
            return ops.conv2d(x, wp, bp, geom, pad=pad, relu=True, residual=res)
        for _ in range(3):
            y = run()
        torch.cuda.synchronize()
        # captured in a graph: eager calls are host-bound (~75 us of Python + binding per call)
        graph = torch.cuda.CUDAGraph()
        s_cap = torch.cuda.Stream()
        with torch.cuda.stream(s_cap):
            with torch.cuda.graph(graph, stream=s_cap):
                for _ in range(a.reps):
                    y = run()
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        graph.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        fl = 2.0 * a.batch * s["H"] ** 2 * s["cout"] * s["cin"] * s["k"] ** 2
        # fp32 oracle (bf16 operands): relative max error of the timed kernel's output
        xr = x.float().permute(0, 3, 1, 2)
        ref = torch.nn.functional.conv2d(xr, w.to(dev).to(torch.bfloat16).float(), b.to(dev),
                                         padding=pad)
        if res is not None:
            ref = ref + res.float().permute(0, 3, 1, 2)
        ref = torch.relu(ref).permute(0, 2, 3, 1)
        err = float((y.float() - ref).abs().max() / ref.abs().max())
        print(json.dumps({"tag": a.tag, "layer": name, "us": round(us, 1), "rel_err": err,
                          "tflops": round(fl / us / 1e6, 1),
                          "checksum": float(y.float().abs().mean())}), flush=True)


if __name__ == "__main__":
    main()
