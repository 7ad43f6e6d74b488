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
from supervised import diagnose, lines, ranks_serving, read_keys, start_job, wait_for

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C = native()
K = C.kafka


_lines = lines


def test_child_argv_drops_ranks():
    assert child_argv(["t", "in", "out", "--ranks", "3", "--stub"]) == ["t", "in", "out",
                                                                       "--stub"]
    assert child_argv(["t", "in", "out", "--ranks=2"]) == ["t", "in", "out"]


def test_supervised_rank_killed_is_respawned_and_rejoins(tmp_path):
    b = K.Broker()
    b.start()
    sup = None
    log = tmp_path / "job.log"
    try:
        b.create_topic("in", 6)
        b.create_topic("out", 1)
        rng = np.random.default_rng(5)
        payload = [C.encode_instances(rng.random((1, 32, 32, 3), dtype=np.float32))
                   for _ in range(16)]
        metrics = tmp_path / "m.jsonl"
        reg = tmp_path / "reg"
        sup = start_job(["sup", "in", "out", "--ranks", "3",
                         "--bootstrap", f"127.0.0.1:{b.port}", "--stub", "--group-membership",
                         "--group-id", "G", "--start-offset", "committed",
                         "--auto-offset-reset", "earliest", "--output-key", "input",
                         "--session-timeout-ms", "1500", "--heartbeat-interval-ms", "100",
                         "--rebalance-timeout-ms", "3000", "--commit-interval-ms", "100",
                         "--rank-restart-backoff-ms", "300", "--rank-max-restarts", "2",
                         "--registry-dir", str(reg), "--metrics-file", str(metrics),
                         "--metrics-interval", "0.25", "--max-batch", "16", "--max-wait-us",
                         "500", "--source-parallelism", "1", "--duration", "120"], log)
        assert wait_for(lambda: ranks_serving(metrics, 3, 6), 90), \
            "three supervised ranks did not take partitions\n" + \
            diagnose(b, {}, [], "G", "in", 6, log, metrics)
        assert wait_for(lambda: (reg / "sup.json").exists() and (reg / "sup.r1.json").exists())
        victim = json.load(open(reg / "sup.r1.json"))["pid"]
        where = {}
        i = 0
        t0 = time.time()
        gen_at_kill = None
        while time.time() - t0 < 5.0:
            for _ in range(6):
                k = f"s{i}".encode()
                where[k] = (i % 6, b.log_end("in", i % 6))
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
        out = {}

        def all_out():
            out.update(read_keys(b, "out"))
            return set(where) <= set(out)

        assert wait_for(all_out, 60), "records were lost across the rank restart\n" + \
            diagnose(b, where, out, "G", "in", 6, log, metrics)
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
        sup.wait(timeout=60)
        err = open(log, errors="replace").read()
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


def _stop_job(sup, reg, name):
    kill = subprocess.run([sys.executable, "-m", "gale", "kill", name, "--wait-secs", "30",
                           "--registry-dir", str(reg)], cwd=ROOT, timeout=60)
    assert kill.returncode == 0
    sup.wait(timeout=60)


def test_supervised_single_rank(tmp_path):
    """--ranks 1: the supervisor holds NAME in the registry, the rank registers as
    NAME.r0 and serves (it used to collide with its own supervisor and exit 1)."""
    b = K.Broker()
    b.start()
    sup = None
    log = tmp_path / "job.log"
    try:
        b.create_topic("in", 1)
        b.create_topic("out", 1)
        metrics = tmp_path / "m.jsonl"
        reg = tmp_path / "reg"
        sup = start_job(["one", "in", "out", "--ranks", "1", "--bootstrap",
                         f"127.0.0.1:{b.port}", "--stub", "--start-offset", "earliest",
                         "--registry-dir", str(reg), "--metrics-file", str(metrics),
                         "--metrics-interval", "0.25", "--duration", "60"], log)
        assert wait_for(lambda: ranks_serving(metrics, 1, 1, group=False), 60), \
            open(log).read()[-3000:]
        assert (reg / "one.json").exists() and (reg / "one.r0.json").exists()
        rng = np.random.default_rng(1)
        for i in range(10):
            b.append("in", 0, [C.encode_instances(rng.random((1, 32, 32, 3), dtype=np.float32))],
                     [b"k%d" % i])
        assert wait_for(lambda: len(b.read("out", 0)) == 10, 30)
        _stop_job(sup, reg, "one")
        assert sup.returncode == 0, open(log).read()[-3000:]
        sup = None
    finally:
        if sup is not None and sup.poll() is None:
            sup.kill()
            sup.wait()
        b.stop()


def test_static_partition_rank_respawn_resumes_from_committed(tmp_path):
    """Static p % world partitions with the default --start-offset latest: a
    respawned rank resumes from the committed offsets (storm-kafka's restarted worker reads its
    ZK offsets), so the records in flight when it was SIGKILLed are served, not skipped."""
    b = K.Broker()
    b.start()
    sup = None
    log = tmp_path / "job.log"
    try:
        b.create_topic("in", 4)
        b.create_topic("out", 1)
        rng = np.random.default_rng(2)
        payload = [C.encode_instances(rng.random((1, 32, 32, 3), dtype=np.float32))
                   for _ in range(8)]
        metrics = tmp_path / "m.jsonl"
        reg = tmp_path / "reg"
        sup = start_job(["st", "in", "out", "--ranks", "2", "--bootstrap",
                         f"127.0.0.1:{b.port}", "--stub", "--output-key", "input",
                         "--commit-interval-ms", "100", "--rank-restart-backoff-ms", "200",
                         "--stub-delay-us", "2000", "--max-batch", "8",
                         "--registry-dir", str(reg), "--metrics-file", str(metrics),
                         "--metrics-interval", "0.25", "--duration", "120"], log)
        assert wait_for(lambda: ranks_serving(metrics, 2, 4, group=False), 60), \
            diagnose(b, {}, [], "st", "in", 4, log, metrics)
        victim = json.load(open(reg / "st.r1.json"))["pid"]
        where = {}
        for i in range(400):
            k = f"t{i}".encode()
            where[k] = (i % 4, b.log_end("in", i % 4))
            b.append("in", i % 4, [payload[i % 8]], [k])
            if i == 200:
                os.kill(victim, signal.SIGKILL)
        out = {}

        def all_out():
            out.update(read_keys(b, "out"))
            return set(where) <= set(out)

        assert wait_for(all_out, 60), diagnose(b, where, out, "st", "in", 4, log, metrics)
        _stop_job(sup, reg, "st")
        sup = None
    finally:
        if sup is not None and sup.poll() is None:
            sup.kill()
            sup.wait()
        b.stop()


def test_delivery_failure_exits_rank_and_respawn_delivers(tmp_path):
    """at-least-once end to end: the output topic rejects every produce for a while and the
    producer's retries run out, so the rank raises delivery_failed, exits non-zero and is
    respawned; the new incarnation resumes from the committed offsets (which never passed the
    undelivered records) and, once the broker accepts produces again, every key has an
    output."""
    b = K.Broker()
    b.start()
    sup = None
    log = tmp_path / "job.log"
    try:
        b.create_topic("in", 2)
        b.create_topic("out", 1)
        rng = np.random.default_rng(3)
        metrics = tmp_path / "m.jsonl"
        reg = tmp_path / "reg"
        sup = start_job(["df", "in", "out", "--ranks", "1", "--bootstrap",
                         f"127.0.0.1:{b.port}", "--stub", "--output-key", "input",
                         "--start-offset", "committed", "--auto-offset-reset", "earliest",
                         "--producer-retries", "2", "--retry-backoff-ms", "20",
                         "--commit-interval-ms", "100", "--rank-restart-backoff-ms", "500",
                         "--rank-max-restarts", "5",
                         "--registry-dir", str(reg), "--metrics-file", str(metrics),
                         "--metrics-interval", "0.25", "--duration", "120"], log)
        assert wait_for(lambda: ranks_serving(metrics, 1, 2, group=False), 60), \
            diagnose(b, {}, [], "df", "in", 2, log, metrics)
        where = {}
        for i in range(40):
            k = f"d{i}".encode()
            where[k] = (i % 2, b.log_end("in", i % 2))
            if i == 20:
                b.fail_produce("out", 1 << 30)  # the broker refuses every produce from here
            b.append("in", i % 2, [C.encode_instances(rng.random((1, 32, 32, 3),
                                                                 dtype=np.float32))], [k])
            time.sleep(0.01)

        def exited():
            return '"rank_exit"' in open(log, errors="replace").read()

        assert wait_for(exited, 60), diagnose(b, where, read_keys(b, "out"), "df", "in", 2, log,
                                              metrics)
        b.fail_produce("out", 0)  # accepting again
        out = {}

        def all_out():
            out.update(read_keys(b, "out"))
            return set(where) <= set(out)

        assert wait_for(all_out, 60), diagnose(b, where, out, "df", "in", 2, log, metrics)
        text = open(log, errors="replace").read()
        assert "at-least-once delivery failed" in text
        events = [json.loads(x) for x in text.splitlines() if x.startswith('{"ts"')]
        assert any(e["event"] == "rank_exit" and e["rc"] == 3 for e in events)
        assert any(e["event"] == "rank_respawn" for e in events)
        _stop_job(sup, reg, "df")
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
