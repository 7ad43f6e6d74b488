"""Rank supervisor: Storm's supervisor daemons restarting dead worker JVMs, for gale's
one-process-per-GPU mode.

In the reference, ``Config.setNumWorkers(8)`` (MainTopology.java:25,65-66) gives the topology 8
worker JVMs, ``StormSubmitter.submitTopology`` (:69) hands them to Nimbus, and each node's
Supervisor respawns a worker that dies; the respawned worker re-runs ``InferenceBolt.prepare()``
and reloads its model. gale's equivalent:

    python -m gale NAME IN OUT --ranks N [--rank-max-restarts R] [--rank-restart-backoff-ms B]

* this process (the supervisor) never touches a GPU: it registers NAME in the topology registry
  (so ``python -m gale kill NAME`` reaches it), starts one CHILD process per rank
  (``python -m gale NAME IN OUT ...`` with RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* set, as
  torchrun would) and waits;
* start-up is all-or-nothing: the first incarnation of every rank rendezvouses, RCCL-broadcasts
  the weights and reports ready. A rank that fails before the whole job is ready (a process-group
  or RCCL init failure, a bad device) ends the job with a non-zero status; nothing waits on a
  rendezvous that cannot complete (``--rank-start-timeout-s`` bounds the wait too);
* after start-up a rank that exits non-zero or is killed by a signal is respawned as a FRESH
  process (never an exec) after ``--rank-restart-backoff-ms``, at most ``--rank-max-restarts``
  times per rank (-1: always, like Storm). The new incarnation materialises the weights itself
  (the seeded init or ``--weights`` file, identical to rank 0's broadcast: ``prepare()``
  reloading the model), takes its partitions again - static ``p % world`` ones, or through the
  Kafka consumer group with ``--group-membership`` (a rebalance moved them to the survivors
  when it died; it rejoins, the generation advances and they come back) - and resumes from the
  committed offsets with ``--start-offset committed``;
* a rank exits 0 when its duration ends or it is told to stop; that is not a failure. A rank
  whose replicas are all dead (a device hung and the watchdog killed them) exits with status 3
  (``topology.RankFailedError``), so it is replaced instead of serving on at zero capacity;
* SIGTERM / SIGINT to the supervisor are forwarded to every rank (graceful drain), and the
  ranks die with it (PR_SET_PDEATHSIG) if it is killed outright.

Every child gets ``GALE_RANK_INCARNATION`` (0, 1, ...), which its metrics lines and
``/metrics`` carry as ``rank_restarts``; the supervisor writes one JSON line per event to
stderr (``rank_start`` / ``rank_exit`` / ``rank_respawn`` / ``rank_abandoned``).
"""

from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import time
from typing import Dict, List, Optional

# exit status of a rank whose replicas are all dead (topology.RankFailedError)
RANK_FAILED = 3


def _pdeathsig():
    """preexec_fn: the child gets SIGTERM when the supervisor dies (PR_SET_PDEATHSIG)."""
    import ctypes

    try:
        ctypes.CDLL(None).prctl(1, signal.SIGTERM, 0, 0, 0)
    except (OSError, AttributeError):
        pass


def child_argv(argv: List[str]) -> List[str]:
    """The rank's command line: the topology arguments minus the supervisor's own --ranks."""
    out, skip = [], False
    for tok in argv:
        if skip:
            skip = False
            continue
        if tok == "--ranks":
            skip = True
            continue
        if tok.startswith("--ranks="):
            continue
        out.append(tok)
    return out


class RankSupervisor:
    """Starts ``n`` rank processes of one topology and keeps them alive (module docstring)."""

    def __init__(self, argv: List[str], n: int, max_restarts: int = 10,
                 backoff_ms: int = 1000, start_timeout_s: float = 300.0,
                 run_dir: str = "", env: Optional[Dict[str, str]] = None,
                 command: Optional[List[str]] = None, log=None):
        if n < 1:
            raise ValueError("--ranks must be >= 1")
        self.argv = child_argv(argv)
        self.n = n
        self.max_restarts = max_restarts
        self.backoff_s = max(0, backoff_ms) / 1e3
        self.start_timeout_s = start_timeout_s
        self.run_dir = run_dir
        self.env = dict(os.environ if env is None else env)
        # the rank program (tests substitute a stand-in)
        self.command = command or [sys.executable, "-m", "gale", *self.argv]
        self.log = log or sys.stderr
        self.procs: List[Optional[subprocess.Popen]] = [None] * n
        self.incarnation = [0] * n
        self.restarts = [0] * n
        self.respawn_at: Dict[int, float] = {}
        self.abandoned = set()
        self.done = set()
        self.stopping = False
        self.master_port = 0

    def _event(self, kind: str, **kw) -> None:
        self.log.write(json.dumps({"ts": round(time.time(), 3), "event": kind, **kw}) + "\n")
        self.log.flush()

    def _ready_path(self, r: int) -> str:
        return os.path.join(self.run_dir, f"rank{r}.ready")

    def _spawn(self, r: int) -> None:
        env = dict(self.env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(self.n),
                   LOCAL_WORLD_SIZE=str(self.n), GROUP_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(self.master_port),
                   GALE_SUPERVISED="1", GALE_RANK_INCARNATION=str(self.incarnation[r]),
                   GALE_READY_FILE=self._ready_path(r), HSA_ENABLE_IPC_MODE_LEGACY="0")
        try:
            os.unlink(self._ready_path(r))
        except FileNotFoundError:
            pass
        self.procs[r] = subprocess.Popen(self.command, env=env, preexec_fn=_pdeathsig)
        self._event("rank_start" if self.incarnation[r] == 0 else "rank_respawn", rank=r,
                    pid=self.procs[r].pid, incarnation=self.incarnation[r])

    def signal_all(self, sig: int) -> None:
        for p in self.procs:
            if p is not None and p.poll() is None:
                try:
                    p.send_signal(sig)
                except ProcessLookupError:
                    pass

    def stop(self, *_):
        """Graceful stop (SIGTERM / SIGINT / kill NAME): forward to every rank."""
        self.stopping = True
        self.signal_all(signal.SIGTERM)

    def _kill_all(self, wait_s: float = 10.0) -> None:
        self.signal_all(signal.SIGTERM)
        deadline = time.monotonic() + wait_s
        for p in self.procs:
            if p is None:
                continue
            try:
                p.wait(max(0.0, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    def startup(self) -> int:
        """Start every rank's first incarnation; 0 once all are ready, else the failing status
        (every rank is then stopped: a partial start-up would hang in the rendezvous)."""
        from gale.utils import free_port

        os.makedirs(self.run_dir, exist_ok=True)
        self.master_port = free_port()
        for r in range(self.n):
            self._spawn(r)
        deadline = time.monotonic() + self.start_timeout_s
        while True:
            if self.stopping:
                self._kill_all()
                return 0
            ready = 0
            for r, p in enumerate(self.procs):
                rc = p.poll()
                if rc is not None:
                    if rc == 0 and os.path.exists(self._ready_path(r)):
                        ready += 1  # (ran and finished already: a very short --duration)
                        continue
                    self._event("startup_failed", rank=r, rc=rc)
                    self._kill_all()
                    return rc if rc > 0 else 128 - rc
                if os.path.exists(self._ready_path(r)):
                    ready += 1
            if ready == self.n:
                self._event("job_ready", ranks=self.n)
                return 0
            if time.monotonic() > deadline:
                self._event("startup_timeout", seconds=self.start_timeout_s)
                self._kill_all()
                return 124
            time.sleep(0.05)

    def monitor(self) -> int:
        """Respawn failed ranks until every rank has finished; the job's exit status."""
        while True:
            now = time.monotonic()
            if self.stopping:  # a rank waiting to be respawned is finished instead
                self.done.update(self.respawn_at)
                self.respawn_at.clear()
            for r, p in enumerate(self.procs):
                if r in self.done or r in self.abandoned or r in self.respawn_at:
                    continue
                rc = p.poll()
                if rc is None:
                    continue
                self._event("rank_exit", rank=r, rc=rc, incarnation=self.incarnation[r])
                if rc == 0 or self.stopping:
                    self.done.add(r)
                elif self.max_restarts < 0 or self.restarts[r] < self.max_restarts:
                    self.respawn_at[r] = now + self.backoff_s
                else:
                    self._event("rank_abandoned", rank=r, restarts=self.restarts[r])
                    self.abandoned.add(r)
            for r, t in list(self.respawn_at.items()):
                if now >= t and not self.stopping:
                    del self.respawn_at[r]
                    self.restarts[r] += 1
                    self.incarnation[r] += 1
                    self._spawn(r)
            if len(self.done) + len(self.abandoned) == self.n:
                self._event("job_exit", restarts=self.restarts, abandoned=sorted(self.abandoned))
                return 1 if self.abandoned else 0
            time.sleep(0.05)

    def run(self) -> int:
        old = {s: signal.signal(s, self.stop) for s in (signal.SIGTERM, signal.SIGINT)}
        try:
            rc = self.startup()
            if rc != 0 or self.stopping:
                return rc
            return self.monitor()
        finally:
            for s, h in old.items():
                signal.signal(s, h)
            self._kill_all()


def run_supervised(cfg, argv: List[str]) -> int:
    """``python -m gale NAME IN OUT --ranks N``: register NAME, supervise N rank processes."""
    import logging
    import tempfile

    from gale.topology import AlreadyAliveError, Registry

    log = logging.getLogger("gale.supervisor")
    registry = Registry(cfg.registry_dir)
    try:
        registry.register(cfg.topology_name, {
            "input_topic": cfg.input_topic, "output_topic": cfg.output_topic,
            "bootstrap": cfg.bootstrap, "model": cfg.model, "ranks": cfg.ranks,
            "role": "supervisor"})
    except AlreadyAliveError as e:  # MainTopology.java:79-80
        log.error("%s", e)
        return 1
    try:
        with tempfile.TemporaryDirectory(prefix=f"gale-{cfg.topology_name}-") as run_dir:
            sup = RankSupervisor(argv, cfg.ranks, cfg.rank_max_restarts,
                                 cfg.rank_restart_backoff_ms, cfg.rank_start_timeout_s,
                                 run_dir=run_dir)
            return sup.run()
    finally:
        registry.unregister(cfg.topology_name)
