"""Process-group bring-up for one-process-per-GPU serving (bench.py, ``torchrun -m gale``).

Every rank drives one GPU; the group exists for the weight broadcast (``weights.py``) and the
bench's max-over-ranks timing. The backend is "nccl" (RCCL over xGMI on ROCm) whenever each
rank owns its own device, and gloo only for the shared-GPU rehearsal (RCCL refuses two ranks on
one device) and the CPU stub engine.
"""

from __future__ import annotations

import os
from datetime import timedelta

import torch
import torch.distributed as dist


def init_rank_group(local_rank: int, use_gpu: bool, shared_gpu: bool = False) -> str:
    """Initialise the default process group from the torchrun env (RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT); returns the backend. ``device_id`` binds the RCCL communicator
    to this rank's GPU eagerly, so a mis-mapped rank fails here and not in the first
    collective."""
    if dist.is_initialized():
        return dist.get_backend()
    # fault injection for the failure-path tests: this rank's group init fails
    if os.environ.get("GALE_FAULT_INIT_RANK", "") == os.environ.get("RANK", "0"):
        raise RuntimeError("injected process-group init failure (GALE_FAULT_INIT_RANK)")
    # bounded: a peer that never arrives fails the rendezvous instead of hanging the job
    timeout = timedelta(seconds=float(os.environ.get("GALE_PG_TIMEOUT_S", "300")))
    nccl = use_gpu and not shared_gpu
    if nccl:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank),
                                timeout=timeout)
    else:
        dist.init_process_group("gloo", timeout=timeout)
    return "nccl" if nccl else "gloo"
