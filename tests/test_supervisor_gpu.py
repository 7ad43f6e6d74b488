"""Rank supervisor with real GPU ranks (gale/supervisor.py; Storm's supervisors respawning dead
worker JVMs, MainTopology.java:25,65-66,69).

``python -m gale NAME IN OUT --ranks 2 --shared-gpu-rehearsal`` on the one-GPU box: two rank
processes serve ResNet-20 on GPU 0 (gloo process group for the weight broadcast). One rank is
SIGKILLed mid-stream; the supervisor respawns it as a fresh process that materialises the
weights itself, rejoins the consumer group and resumes from the committed offsets, so every input
record gets a prediction record (a real 10-class softmax)."""

import json
import os
import signal
import subprocess
import sys
import time

import numpy as np
import pytest

from supervised import ROOT, diagnose, lines, ranks_serving, read_keys, start_job, wait_for

pytestmark = pytest.mark.gpu


def test_supervised_gpu_rank_killed_is_respawned(tmp_path):
    """Round-5 driver failure ("records were lost across the GPU rank restart"): the appends
    began once describe_group listed two members, i.e. while the group was still rebalancing,
    before either rank had sought its partitions; with no committed offset yet a fresh group
    starts at the log end (auto.offset.reset=latest), so records appended in that gap were
    never read. Now the appends wait until both ranks report their partitions assigned in one
    generation, the group falls back to the log start (--auto-offset-reset earliest), and
    stderr goes to a file (a pipe that fills blocks the ranks)."""
    from gale._native import native

    C = native()
    K = C.kafka
    b = K.Broker()
    b.start()
    sup = None
    log = tmp_path / "job.log"
    try:
        b.create_topic("in", 4)
        b.create_topic("out", 1)
        rng = np.random.default_rng(7)
        payload = [C.encode_instances(rng.random((1, 32, 32, 3), dtype=np.float32))
                   for _ in range(8)]
        metrics = tmp_path / "m.jsonl"
        reg = tmp_path / "reg"
        sup = start_job(["gsup", "in", "out", "--ranks", "2",
                         "--shared-gpu-rehearsal", "--model", "resnet20", "--replicas", "1",
                         "--bootstrap", f"127.0.0.1:{b.port}", "--group-membership",
                         "--group-id", "GG", "--start-offset", "committed",
                         "--auto-offset-reset", "earliest", "--output-key", "input",
                         "--session-timeout-ms", "2000", "--heartbeat-interval-ms", "100",
                         "--rebalance-timeout-ms", "4000", "--commit-interval-ms", "100",
                         "--rank-restart-backoff-ms", "200", "--rank-max-restarts", "2",
                         "--rank-start-timeout-s", "90", "--no-numa-pin",
                         "--registry-dir", str(reg), "--metrics-file", str(metrics),
                         "--metrics-interval", "0.25", "--max-batch", "16", "--max-wait-us",
                         "500", "--source-parallelism", "1", "--duration", "100"], log)
        assert wait_for(lambda: ranks_serving(metrics, 2, 4), 90, 0.1), \
            "two supervised GPU ranks did not both take partitions\n" + \
            diagnose(b, {}, [], "GG", "in", 4, log, metrics)
        assert wait_for(lambda: (reg / "gsup.r1.json").exists(), 10)
        victim = json.load(open(reg / "gsup.r1.json"))["pid"]
        where, i, gen_at_kill = {}, 0, None
        t0 = time.time()
        while time.time() - t0 < 3.0:
            for _ in range(4):
                k = f"g{i}".encode()
                p = i % 4
                where[k] = (p, b.log_end("in", p))
                b.append("in", p, [payload[i % 8]], [k])
                i += 1
            if gen_at_kill is None and time.time() - t0 > 1.0:
                gen_at_kill = b.describe_group("GG")["generation"]
                os.kill(victim, signal.SIGKILL)
            time.sleep(0.02)

        def respawned():
            rows = [r for r in lines(metrics) if r.get("rank") == 1
                    and r.get("rank_restarts") == 1]
            return rows and rows[-1].get("assigned_partitions", 0) > 0 \
                and rows[-1].get("generation", -1) > gen_at_kill

        assert wait_for(respawned, 60, 0.1), lines(metrics)[-4:]
        assert json.load(open(reg / "gsup.r1.json"))["pid"] != victim
        out = {}

        def all_out():
            out.update(read_keys(b, "out"))
            return set(where) <= set(out)

        assert wait_for(all_out, 60, 0.1), "records were lost across the GPU rank restart\n" + \
            diagnose(b, where, out, "GG", "in", 4, log, metrics)
        for k in list(where)[:: max(1, len(where) // 20)]:
            p = np.array(json.loads(out[k])["predictions"], dtype=np.float64)
            assert p.shape == (1, 10) and abs(p.sum() - 1.0) < 1e-3
        kill = subprocess.run([sys.executable, "-m", "gale", "kill", "gsup", "--wait-secs", "30",
                               "--registry-dir", str(reg)], cwd=ROOT, timeout=60)
        assert kill.returncode == 0
        sup.wait(timeout=60)
        err = open(log, errors="replace").read()
        assert sup.returncode == 0, err[-3000:]
        events = [json.loads(x) for x in err.splitlines() if x.startswith('{"ts"')]
        assert ("rank_respawn", 1) in [(e["event"], e.get("rank")) for e in events]
        sup = None
    finally:
        if sup is not None and sup.poll() is None:
            sup.kill()
            sup.wait()
        b.stop()
