"""Time the GPU prediction-text kernel (format.hip) on softmax-like rows."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gale._native import native  # noqa: E402

C = native()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2560
rng = np.random.default_rng(0)
z = rng.normal(size=(n // 10, 10)).astype(np.float32) * 4
e = np.exp(z - z.max(axis=1, keepdims=True))
x = torch.from_numpy((e / e.sum(axis=1, keepdims=True)).astype(np.float32).ravel()).cuda()
out = torch.empty((x.numel(), 16), dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for _ in range(5):
    C.format_floats_java(x.numel(), x.data_ptr(), out.data_ptr(), s)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(50):
    C.format_floats_java(x.numel(), x.data_ptr(), out.data_ptr(), s)
b.record()
torch.cuda.synchronize()
print(json.dumps({"values": x.numel(), "us_per_call": a.elapsed_time(b) * 1000 / 50}))
