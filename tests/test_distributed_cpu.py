"""Multi-process paths on CPU (gloo, world_size 2): the weight broadcast that replaces every
InferenceBolt loading its own model copy (InferenceBolt.java:48-58; RCCL over xGMI on GPUs) and
bench.py's one-process-per-GPU launch contract (torch.distributed.run, max-over-ranks timing)."""

import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():  # (kept local: the spawned workers import nothing from gale first)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bcast_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gale.models import get_model
    from gale.parallel.weights import materialize_weights

    net = get_model("resnet20")
    # only rank 0's seed matters: every other rank receives rank 0's buffer
    buf = materialize_weights(net, torch.device("cpu"), seed=0 if rank == 0 else 99)
    q.put((rank, int(buf.sum().item()), buf.numel()))
    dist.destroy_process_group()


def test_weight_broadcast_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert res[0][1:] == res[1][1:]


def test_bench_stub_torchrun_world2():
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
           "--stub", "--steps", "4", "--warmup", "1", "--batch", "32", "--distinct", "64",
           "--replicas-per-gpu", "4", "--step-images", "512", "--min-warmup-s", "0.2",
           "--timeout", "120"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    r = lines[0]
    assert r["n_gpus"] == 2 and r["steps"] == 4 and r["value"] > 0
    # a step = one 32-image micro-batch per replica (4 per GPU by default), on both ranks
    assert r["config"]["parallelism"] == "dp2" and r["config"]["global_batch"] == 512 * 2
    # one input topic shared by the two ranks' broker cluster, one partition per replica
    assert r["config"]["partitions"] == 8
    assert r["step_rate_spread"]["min"] > 0 and r["timed_s"] > 0


def test_bench_plain_entry_launches_ranks():
    """The driver's plain ``python bench.py --gpus 2`` (no torchrun around it): bench.py starts
    one rank per GPU itself (a torch.distributed.run child) and rank 0 reports n_gpus = 2."""
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--stub", "--steps", "3", "--warmup", "1",
           "--batch", "32", "--distinct", "64", "--replicas-per-gpu", "2",
           "--step-images", "256", "--min-warmup-s", "0.2", "--stub-null", "--timeout", "120"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300,
                         env=dict(env, OMP_NUM_THREADS="1"))
    assert out.returncode == 0, out.stderr[-3000:]
    (r,) = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert r["n_gpus"] == 2 and r["config"]["processes"] == 2
    assert r["config"]["parallelism"] == "dp2"
    assert r["config"]["launcher"].startswith("torch.distributed.run child")


def test_bench_plain_entry_too_many_gpus_fails():
    """More GPUs than visible (none here) fails loudly instead of silently running fewer."""
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1"], cwd=ROOT,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "GPU(s) visible" in out.stderr
    assert not [x for x in out.stdout.splitlines() if x.startswith("{")]


def test_bench_stub_rate_mode():
    """bench.py --rate: the open-loop feeder offers a fixed image rate; the engine keeps up, so
    the achieved rate matches the offer and the load is reported in the JSON line."""
    cmd = [sys.executable, "bench.py", "--stub", "--stub-null", "--steps", "20", "--warmup", "2",
           "--step-images", "128", "--min-warmup-s", "0.2", "--distinct", "256",
           "--batch", "16", "--replicas-per-gpu", "2", "--rate", "3000", "--max-wait-us", "500",
           "--timeout", "120"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert out.returncode == 0, out.stderr[-3000:]
    (r,) = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert r["load"].startswith("offered 3000")
    assert 0.7 * 3000 < r["value"] < 1.3 * 3000
    assert r["p50_latency_ms"] < 50


def test_scaling_driver_stub_1_2():
    """tools/scaling.py: bench.py at N = 1 (plain process) and N = 2 (torch.distributed.run,
    gloo stub ranks), one JSON line per N and a summary with the weak-scaling efficiency."""
    cmd = [sys.executable, "tools/scaling.py", "--gpus", "1,2", "--stub", "--steps", "4",
           "--warmup", "1", "--timeout", "240", "--placements", "floating", "--",
           "--batch", "32", "--distinct", "64",
           "--step-images", "512", "--min-warmup-s", "0.2",
           "--replicas-per-gpu", "2", "--stub-null", "--timeout", "120"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600,
                         env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert [r["n_gpus"] for r in lines[:2]] == [1, 2]
    sc = lines[-1]["scaling"]["floating"]
    assert set(sc) == {"1", "2"} and sc["1"]["efficiency"] == 1.0 and sc["2"]["efficiency"] > 0
    assert [x["rank"] for x in sc["2"]["per_rank"]] == [0, 1]
    assert all(x["cores"] is not None and x["img_s"] > 0 for x in sc["2"]["per_rank"])


def test_scaling_driver_single_process_mode():
    """tools/scaling.py --mode single-process: ONE bench.py process drives N "GPUs" (stub
    replicas in N locality slots) - the single-process multi-GPU serving mode."""
    cmd = [sys.executable, "tools/scaling.py", "--gpus", "1,2", "--stub", "--steps", "4",
           "--warmup", "1", "--timeout", "240", "--mode", "single-process", "--",
           "--batch", "32", "--distinct", "64", "--step-images", "512", "--min-warmup-s", "0.2",
           "--replicas-per-gpu", "2", "--stub-null", "--timeout", "120"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600,
                         env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert [r["n_gpus"] for r in lines[:2]] == [1, 2]
    assert lines[1]["config"]["processes"] == 1 and lines[1]["config"]["partitions"] == 4
    assert lines[-1]["mode"] == "single-process"


def _bench_stub(n, extra=(), env_extra=None, timeout=300):
    cmd = [sys.executable, "bench.py", "--gpus", str(n), "--stub", "--steps", "3", "--warmup",
           "1", "--batch", "32", "--distinct", "64", "--replicas-per-gpu", "2",
           "--step-images", "256", "--min-warmup-s", "0.2", "--stub-null", "--timeout", "120",
           *extra]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    return subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                          env=dict(env, OMP_NUM_THREADS="1", **(env_extra or {})))


def test_bench_plain_entry_world4_per_rank_view():
    """The driver's ``python bench.py --gpus 4`` at world 4 (gloo stub ranks): every rank leads
    and consumes its own input partitions (p % 4 == rank), produces to its own output partition,
    the reported window is the slowest rank's and ``value`` the sum over ranks / that window."""
    out = _bench_stub(4)
    assert out.returncode == 0, out.stderr[-3000:]
    (r,) = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert r["n_gpus"] == 4 and r["config"]["processes"] == 4
    assert r["config"]["parallelism"] == "dp4" and r["config"]["partitions"] == 8
    ranks = r["ranks"]
    assert [x["rank"] for x in ranks] == [0, 1, 2, 3]
    for x in ranks:
        assert x["partitions"] == [p for p in range(8) if p % 4 == x["rank"]]
        assert x["output_partition"] == x["rank"]
        assert x["images"] >= 3 * 256
    assert r["timed_s"] == pytest.approx(max(x["timed_s"] for x in ranks), abs=2e-3)
    total = sum(x["images"] for x in ranks)
    assert r["value"] == pytest.approx(total / max(x["timed_s"] for x in ranks), rel=2e-3)


def test_bench_rank_init_failure_fails_the_job_fast():
    """A rank whose process-group init fails (injected in rank 2 of 3) makes the whole
    ``bench.py --gpus 3`` exit non-zero promptly: no rank is left hanging in the rendezvous and
    no JSON line is printed."""
    import time

    t0 = time.time()
    out = _bench_stub(3, env_extra={"GALE_FAULT_INIT_RANK": "2", "GALE_PG_TIMEOUT_S": "60"},
                      timeout=240)
    assert out.returncode != 0
    assert "injected process-group init failure" in out.stderr
    assert not [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert time.time() - t0 < 120


def test_scaling_dry_run_prints_per_n_config():
    """tools/scaling.py --dry-run: the command and per-rank config of every N, nothing run; the
    N = 1 sizing is pinned for every larger N (weak scaling at equal per-GPU work)."""
    out = subprocess.run([sys.executable, "tools/scaling.py", "--gpus", "1,2,4,8", "--dry-run"],
                         cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    # N = 1 once, every N > 1 under both host placements (floating, then --rank-slices)
    assert [(r["n_gpus"], r["placement"]) for r in lines] == [
        (1, "floating"), (2, "floating"), (2, "slices"), (4, "floating"), (4, "slices"),
        (8, "floating"), (8, "slices")]
    one = lines[0]["config"]
    for r in lines[1:]:
        assert f"--gpus {r['n_gpus']}" in r["cmd"]
        assert ("--rank-slices" in r["cmd"]) == (r["placement"] == "slices")
        c = r["config"]
        assert c["processes"] == r["n_gpus"]
        for k in ("replicas_per_gpu", "partitions_per_gpu", "decode_threads",
                  "step_images_per_gpu"):
            assert c[k] == one[k], k


def test_scaling_placement_verdict():
    """The sweep's placement decision: --rank-slices becomes the default only when it beats the
    floating placement by more than 2 % at the largest N both ran."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import scaling

    assert scaling.plan([1, 2, 8], ["floating", "slices"]) == [
        (1, "floating"), (2, "floating"), (2, "slices"), (8, "floating"), (8, "slices")]
    res = {"floating": {1: {"value": 2.0}, 2: {"value": 4.0}, 8: {"value": 12.0}},
           "slices": {1: {"value": 2.0}, 2: {"value": 3.9}, 8: {"value": 13.0}}}
    v = scaling.placement_verdict(res)
    assert v["n_gpus"] == 8 and v["faster"] == "slices" and v["default"] == "slices"
    res["slices"][8]["value"] = 12.1  # < 2 %: keep floating
    assert scaling.placement_verdict(res)["default"] == "floating"
    assert scaling.placement_verdict({"floating": res["floating"]}) == {}
