"""Weight materialisation for data-parallel replicas.

The reference has every InferenceBolt task copy ``model/saved_model.pb`` out of the jar and load
its own copy (InferenceBolt.java:48-58). gale initialises (or loads) the packed parameter buffer
once on the source rank and broadcasts it over RCCL (xGMI) to every other GPU in ONE collective:
the buffer layout depends only on the architecture (``param_layout``), so receivers allocate it
without knowing any values.
"""

from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from gale.models.graph import (Network, fold_params, init_params, pack_params, param_layout,
                               unfolded_params)


def host_packed_params(net: Network, seed: int = 0, wdtype: str = "bf16",
                       params: Optional[dict] = None, fold_bn: bool = True) -> torch.Tensor:
    if params is None:
        params = init_params(net, seed=seed)
    if not fold_bn:
        return pack_params(net, unfolded_params(net, params), wdtype, fold_bn=False)
    return pack_params(net, fold_params(net, params), wdtype)


def materialize_weights(net: Network, device: torch.device, seed: int = 0, wdtype: str = "bf16",
                        src: int = 0, group=None, params: Optional[dict] = None,
                        fold_bn: bool = True) -> torch.Tensor:
    """Return the packed parameter buffer on ``device``, identical on every rank of ``group``."""
    _, total = param_layout(net, wdtype, fold_bn)
    distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    rank = dist.get_rank() if distributed else src
    if rank == src:
        buf = host_packed_params(net, seed, wdtype, params, fold_bn).to(device)
    else:
        buf = torch.empty(total, dtype=torch.uint8, device=device)
    if distributed:
        dist.broadcast(buf, src=src, group=group)  # RCCL over xGMI with the "nccl" backend
    return buf


def replicate_weights(src: torch.Tensor, devices: List[int]) -> List[torch.Tensor]:
    """One copy of the packed buffer per device of THIS process: an in-process RCCL
    communicator (ncclCommInitAll) broadcasts it from ``src``'s device over xGMI
    (csrc/comm/rccl.cpp). ``src``'s device must be one of ``devices`` (the root)."""
    from gale._native import native

    root = devices.index(src.device.index or 0)
    out = [src if i == root else torch.empty_like(src, device=torch.device("cuda", d))
           for i, d in enumerate(devices)]
    comm = native().comm.CommGroup(list(devices))
    comm.broadcast(src.data_ptr(), [t.data_ptr() for t in out], src.numel(), root)
    return out
