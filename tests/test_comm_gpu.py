"""In-process RCCL communicator (csrc/comm/rccl.cpp): ncclCommInitAll over the process's GPUs
and a grouped ncclBroadcast of the packed weights (single-process multi-GPU serving). On a
1-GPU box the communicator has one rank: the same RCCL code path, checked byte for byte."""

import pytest
import torch

from gale._native import native
from gale.models import get_model
from gale.parallel.weights import materialize_weights, replicate_weights

pytestmark = pytest.mark.gpu


def test_rccl_broadcast_byte_identity():
    n = torch.cuda.device_count()
    devs = list(range(n))
    g = native().comm.CommGroup(devs)
    assert g.size == n and list(g.devices) == devs
    src = torch.randint(0, 256, (3 << 20,), dtype=torch.uint8, device="cuda:0")
    dst = [torch.zeros_like(src, device=f"cuda:{d}") for d in devs]
    g.broadcast(src.data_ptr(), [t.data_ptr() for t in dst], src.numel(), 0)
    for t in dst:
        assert torch.equal(t.cpu(), src.cpu())


def test_rccl_all_reduce_counters():
    n = torch.cuda.device_count()
    g = native().comm.CommGroup(list(range(n)))
    bufs = [torch.full((4,), float(d + 1), dtype=torch.float64, device=f"cuda:{d}")
            for d in range(n)]
    g.all_reduce_sum_f64([b.data_ptr() for b in bufs], 4)
    want = float(sum(range(1, n + 1)))
    assert all(torch.all(b.cpu() == want) for b in bufs)


def test_replicate_weights_over_rccl():
    net = get_model("resnet20")
    src = materialize_weights(net, torch.device("cuda", 0), seed=3)
    devs = list(range(torch.cuda.device_count()))
    bufs = replicate_weights(src, devs)
    assert [b.device.index for b in bufs] == devs
    for b in bufs:
        assert torch.equal(b.cpu(), src.cpu())


_RANK_SCRIPT = r"""
import torch, torch.distributed as dist
from gale.models import get_model
from gale.parallel.group import init_rank_group
from gale.parallel.weights import materialize_weights
backend = init_rank_group(0, use_gpu=True)
assert backend == "nccl" and dist.get_backend() == "nccl", backend
net = get_model("resnet20")
buf = materialize_weights(net, torch.device("cuda", 0), seed=5)
ref = buf.clone()
dist.broadcast(buf, src=0)          # the weight broadcast bench.py / topology.py issue
mx = torch.tensor([3.5], dtype=torch.float64, device="cuda")
dist.all_reduce(mx, op=dist.ReduceOp.MAX)   # bench.py's max-over-ranks timing
dist.barrier()
torch.cuda.synchronize()
assert torch.equal(buf.cpu(), ref.cpu()) and mx.item() == 3.5
dist.destroy_process_group()
print("RANK_GROUP_OK")
"""


def test_rank_process_group_is_rccl():
    """The per-process ranks' group (gale/parallel/group.py, used by bench.py and
    ``torchrun -m gale``) comes up on the "nccl" backend (RCCL) bound to the rank's GPU, and the
    broadcast / MAX all-reduce / barrier the bench issues complete. World 1 here (RCCL refuses two
    ranks on one device); the same code runs per rank at N > 1."""
    import os
    import socket
    import subprocess
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _RANK_SCRIPT], env=env, cwd=repo,
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "RANK_GROUP_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
