"""A model replica: packed weights resident on one GPU + the native plan executor.

Replaces one InferenceBolt task (InferenceBolt.java:43-62 prepare / :70-99 execute): the model is
materialised once per replica, and each micro-batch is a single hipGraph replay of the whole
forward on the replica's compute stream (graphs captured per batch bucket and I/O slot).
"""

from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch

from gale._native import native
from gale.models.graph import Network, act_scales_from_packed, build_plan


class ModelReplica:
    def __init__(self, net: Network, packed: torch.Tensor, max_batch: int = 256, slots: int = 2,
                 buckets: Optional[Sequence[int]] = None, wdtype: str = "bf16",
                 fused: bool = True, fold_bn: bool = True,
                 chunk: Optional[Tuple[int, int]] = None, fuse_blocks: Optional[bool] = None):
        if not packed.is_cuda:
            raise RuntimeError("ModelReplica needs the packed weights on a GPU")
        self.net = net
        self.packed = packed  # keeps the weights alive
        self.device = packed.device
        self.wdtype = wdtype
        self.act_scales = act_scales_from_packed(net, packed) if wdtype == "fp8" else None
        # chunk = (leading layers, images per chunk): those layers' ops run per chunk of images
        # (PlanSpec::chunk_ops, executor.h), the rest over the whole batch
        cl, ci = chunk if chunk is not None else (0, 0)
        ops, buf_bytes = build_plan(net, packed.data_ptr(), wdtype, self.act_scales, fused=fused,
                                    fold_bn=fold_bn, chunk_layers=cl if ci > 0 else 0,
                                    fuse_blocks=fuse_blocks)
        co = sum(1 for op in ops if op.get("layer", len(net.layers)) < cl) if ci > 0 else 0
        self.ops = ops
        self.buf_bytes = buf_bytes
        self.executor = native().Executor(packed.device.index or 0, ops, buf_bytes, max_batch,
                                          slots, list(buckets or []), co, ci)

    @property
    def max_batch(self) -> int:
        return self.executor.max_batch

    def capture(self) -> int:
        """Pre-capture the hipGraph of every (batch bucket, I/O slot); returns the graph count."""
        with torch.cuda.device(self.device):
            self.executor.capture_all(torch.cuda.current_stream().cuda_stream)
        return self.executor.graphs_captured

    def infer(self, x: torch.Tensor, use_graph: bool = True, slot: int = 0) -> torch.Tensor:
        """x: [B,H,W,C] fp32 (any device) -> softmax [B, classes] fp32 on this replica's GPU."""
        B = x.shape[0]
        if tuple(x.shape[1:]) != tuple(self.net.input_shape):
            raise ValueError(f"input shape {tuple(x.shape[1:])} != {self.net.input_shape}")
        if B > self.max_batch:
            raise ValueError(f"batch {B} > max_batch {self.max_batch}")
        C = native()
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream().cuda_stream
            xd = x.to(self.device, torch.float32).contiguous()
            C.memcpy_async(self.executor.input_ptr(slot), xd.data_ptr(), xd.numel() * 4, stream)
            self.executor.run(slot, B, stream, use_graph)
            out = torch.empty(B, self.net.classes, device=self.device, dtype=torch.float32)
            C.memcpy_async(out.data_ptr(), self.executor.output_ptr(slot), out.numel() * 4, stream)
            return out

    def infer_eager(self, x: torch.Tensor) -> torch.Tensor:
        """Eager launch on caller buffers (no graph, no slot buffers)."""
        with torch.cuda.device(self.device):
            xd = x.to(self.device, torch.float32).contiguous()
            out = torch.empty(x.shape[0], self.net.classes, device=self.device, dtype=torch.float32)
            self.executor.run_on(x.shape[0], xd.data_ptr(), out.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
            return out
