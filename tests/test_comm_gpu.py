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

