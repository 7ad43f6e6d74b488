"""Rank supervisor (gale/supervisor.py): Storm's supervisors respawning dead worker JVMs
(MainTopology.java:25,65-66,69), on CPU with stub replicas.

``python -m gale NAME IN OUT --ranks 3`` starts three rank processes; one is SIGKILLed
mid-stream. The supervisor respawns it as a fresh process, the new incarnation rejoins the
consumer group (the generation advances and it owns partitions again) and, with
``--start-offset committed``, every input record ends up with an output record."""

import json
import os
import signal
import subprocess
import sys
import time

import numpy as np
import pytest

from gale._native import native
from gale.supervisor import RankSupervisor, child_argv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C = native()
K = C.kafka


def wait_for(pred, timeout=30.0):
    t = time.time() + timeout
    while time.time() < t:
        if pred():
            return True
        time.sleep(0.05)
    return False


def _lines(path):
    if not os.path.exists(path):
        return []
    out = []
    for x in open(path):
        x = x.strip()
        if x:
            try:
                out.append(json.loads(x))
            except json.JSONDecodeError:  # (a line being written)
                pass
    return out


def test_child_argv_drops_ranks():
    assert child_argv(["t", "in", "out", "--ranks", "3", "--stub"]) == ["t", "in", "out",
                                                                       "--stub"]
    assert child_argv(["t", "in", "out", "--ranks=2"]) == ["t", "in", "out"]


def test_supervised_rank_killed_is_respawned_and_rejoins(tmp_path):
    b = K.Broker()
    b.start()
    sup = None
    try:
        b.create_topic("in", 6)
        b.create_topic("out", 1)
        rng = np.random.default_rng(5)
        payload = [C.encode_instances(rng.random((1, 32, 32, 3), dtype=np.float32))
                   for _ in range(16)]
        metrics = tmp_path / "m.jsonl"
        cmd = [sys.executable, "-m", "gale", "sup", "in", "out", "--ranks", "3",
               "--bootstrap", f"127.0.0.1:{b.port}", "--stub", "--group-membership",
               "--group-id", "G", "--start-offset", "committed", "--output-key", "input",
               "--session-timeout-ms", "1500", "--heartbeat-interval-ms", "100",
               "--rebalance-timeout-ms", "3000", "--commit-interval-ms", "100",
               "--rank-restart-backoff-ms", "300", "--rank-max-restarts", "2",
               "--registry-dir", str(tmp_path / "reg"), "--metrics-file", str(metrics),
               "--metrics-interval", "0.25", "--max-batch", "16", "--max-wait-us", "500",
               "--source-parallelism", "1", "--duration", "120"]
        sup = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                               text=True, env=dict(os.environ, OMP_NUM_THREADS="1"))
        assert wait_for(lambda: len(b.describe_group("G")["members"]) == 3, 90), \
            "three supervised ranks did not join the group"
        reg = tmp_path / "reg"
        assert wait_for(lambda: (reg / "sup.json").exists() and (reg / "sup.r1.json").exists())
        victim = json.load(open(reg / "sup.r1.json"))["pid"]
        keys = []
        i = 0
        t0 = time.time()
        gen_at_kill = None
        while time.time() - t0 < 5.0:
            for _ in range(6):
                k = f"s{i}".encode()
                keys.append(k)
                b.append("in", i % 6, [payload[i % 16]], [k])
                i += 1
            if gen_at_kill is None and time.time() - t0 > 1.5:
                gen_at_kill = b.describe_group("G")["generation"]
                os.kill(victim, signal.SIGKILL)
            time.sleep(0.02)

        def respawned():
            rows = [r for r in _lines(metrics) if r.get("rank") == 1
                    and r.get("rank_restarts") == 1]
            return rows and rows[-1].get("assigned_partitions", 0) > 0 \
                and rows[-1].get("generation", -1) > gen_at_kill

        assert wait_for(respawned, 60), _lines(metrics)[-6:]
        new_pid = json.load(open(reg / "sup.r1.json"))["pid"]
        assert new_pid != victim
        assert wait_for(lambda: len(b.describe_group("G")["members"]) == 3, 30)
        # at-least-once across the kill: every input key has an output record
        assert wait_for(lambda: set(keys) <= {r["key"] for r in b.read("out", 0)}, 60), \
            "records were lost across the rank restart"
        # the three members of the final generation cover every partition
        g = b.describe_group("G")["generation"]

        def covered():
            last = {}
            for r in _lines(metrics):
                last[r["rank"]] = r
            return len(last) == 3 and all(r.get("generation") == g for r in last.values()) \
                and set().union(*(r["partitions"] for r in last.values())) == set(range(6))

        assert wait_for(covered, 30)
        kill = subprocess.run([sys.executable, "-m", "gale", "kill", "sup", "--wait-secs", "30",
                               "--registry-dir", str(reg)], cwd=ROOT, timeout=60)
        assert kill.returncode == 0
        _, err = sup.communicate(timeout=60)
        assert sup.returncode == 0, err[-3000:]
        events = [json.loads(x) for x in err.splitlines() if x.startswith('{"ts"')]
        kinds = [(e["event"], e.get("rank")) for e in events]
        assert ("rank_respawn", 1) in kinds and ("job_ready", None) in kinds
        ex = [e for e in events if e["event"] == "rank_exit" and e["rank"] == 1]
        assert ex[0]["rc"] == -signal.SIGKILL
        assert [e for e in events if e["event"] == "job_exit"][0]["restarts"] == [0, 1, 0]
        sup = None
    finally:
        if sup is not None and sup.poll() is None:
            sup.kill()
            sup.wait()
        b.stop()


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(body)
    return p


def test_startup_failure_of_one_rank_ends_the_job(tmp_path):
    """A rank that fails before the job is ready (e.g. its process-group / RCCL init) ends the
    whole job with a non-zero status; the other ranks (stuck waiting for it) are stopped."""
    body = ("import os, sys, time\n"
            "if os.environ['RANK'] == '1':\n"
            "    sys.exit(7)\n"
            "time.sleep(60)\n")
    script = _script(tmp_path, body)
    # a stand-in rank program instead of python -m gale
    s = RankSupervisor([], 3, run_dir=str(tmp_path / "run"), log=open(os.devnull, "w"),
                       command=[sys.executable, str(script)])
    t0 = time.time()
    rc = s.run()
    assert rc == 7
    assert time.time() - t0 < 30
    assert all(p.poll() is not None for p in s.procs)


def test_respawn_budget_and_clean_exit(tmp_path):
    """After start-up a failing rank is respawned up to the budget and then abandoned (job
    status 1); ranks that finish with status 0 are not respawned."""
    body = ("import os, sys, time, json\n"
            "json.dump({}, open(os.environ['GALE_READY_FILE'], 'w'))\n"
            "time.sleep(0.3)\n"
            "sys.exit(3 if os.environ['RANK'] == '0' else 0)\n")
    script = _script(tmp_path, body)
    log = tmp_path / "events.jsonl"
    s = RankSupervisor([], 2, max_restarts=2, backoff_ms=50, run_dir=str(tmp_path / "run"),
                       log=open(log, "w"), command=[sys.executable, str(script)])
    rc = s.run()
    assert rc == 1
    assert s.restarts == [2, 0]
    ev = [json.loads(x) for x in open(log)]
    assert [e["incarnation"] for e in ev if e["event"] == "rank_respawn"] == [1, 2]
    assert any(e["event"] == "rank_abandoned" and e["rank"] == 0 for e in ev)


@pytest.mark.parametrize("sig", [signal.SIGTERM])
def test_supervisor_forwards_stop(tmp_path, sig):
    body = ("import os, signal, sys, time, json\n"
            "signal.signal(signal.SIGTERM, lambda *_: sys.exit(0))\n"
            "json.dump({}, open(os.environ['GALE_READY_FILE'], 'w'))\n"
            "time.sleep(60)\n")
    script = _script(tmp_path, body)
    s = RankSupervisor([], 2, run_dir=str(tmp_path / "run"), log=open(os.devnull, "w"),
                       command=[sys.executable, str(script)])
    import threading

    threading.Timer(1.5, lambda: s.stop()).start()
    t0 = time.time()
    rc = s.run()
    assert rc == 0 and time.time() - t0 < 20
    assert all(p.returncode == 0 for p in s.procs)


def test_rank_with_every_replica_dead_exits_3(tmp_path):
    """A rank that can no longer serve (every replica dead, none being restarted) exits with
    status 3 instead of running on at zero capacity, so the supervisor replaces it."""
    b = K.Broker()
    b.start()
    try:
        b.create_topic("in", 1)
        b.create_topic("out", 1)
        rng = np.random.default_rng(6)
        for i in range(64):
            b.append("in", 0, [C.encode_instances(rng.random((1, 32, 32, 3),
                                                             dtype=np.float32))], [b"k%d" % i])
        cmd = [sys.executable, "-m", "gale", "dead", "in", "out", "--bootstrap",
               f"127.0.0.1:{b.port}", "--stub", "--replicas", "1", "--max-restarts", "0",
               "--fault", "replica_crash@2", "--restart-backoff-ms", "100",
               "--start-offset", "earliest", "--max-batch", "4", "--duration", "60",
               "--registry-dir", str(tmp_path / "reg"), "--metrics-interval", "0"]
        t0 = time.time()
        p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=90,
                           env=dict(os.environ, OMP_NUM_THREADS="1"))
        assert p.returncode == 3, p.stderr[-2000:]
        assert "every replica is dead" in p.stderr
        assert time.time() - t0 < 45
    finally:
        b.stop()
