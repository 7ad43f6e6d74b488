"""``python -m gale`` — the MainTopology command line (R1) plus operational subcommands.

    python -m gale <TOPOLOGY_NAME> <INPUT_TOPIC> <OUTPUT_TOPIC> [--bootstrap H:P] [options]
        Run a topology (the reference's ``storm jar ... dke.model.MainTopology NAME IN OUT``,
        README.md:54-58, MainTopology.java:32-42). Unlike the reference, the Kafka address is a
        flag (the reference hard-codes empty zkHosts/bootstrap strings, :33-34) and every
        parallelism constant of :25-28 is an option. Runs for --duration seconds (reference: 1 h)
        or until ``python -m gale kill NAME`` / SIGTERM.
    python -m gale kill <NAME> [--wait-secs S]   (KillOptions wait_secs, :73-77)
    python -m gale list
    python -m gale broker [--port 9092] [--partitions N]     embedded Kafka-protocol broker
    python -m gale produce <TOPIC> [--images N] [--model M] [--rate R]   synthetic InstObj load
    python -m gale consume <TOPIC> [--max N] [--from-beginning]          print output records

``--profile DIR`` re-runs the topology under ``rocprofv3 --kernel-trace --marker-trace --stats``
(roctx ranges on every host pipeline stage, ``--trace``); ``GALE_ROCTX=1`` turns the ranges on
for an externally launched profiler.

Multi-GPU, one process per GPU: ``python -m gale NAME IN OUT --ranks 8`` starts and supervises
one rank process per GPU and respawns a rank that dies (Storm's supervisors, gale/supervisor.py);
``python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m gale NAME IN OUT
...`` runs the same ranks without respawning. Rank r consumes the input partitions
p % WORLD_SIZE == r (or its consumer-group share) and weights are RCCL-broadcast from rank 0.
"""

from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time
from dataclasses import fields
from typing import List, Optional

from gale.config import CHOICES, GaleConfig, from_sources

SUBCOMMANDS = ("kill", "list", "broker", "produce", "consume")


def _topology_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(
        prog="python -m gale",
        description="Run a gale streaming-inference topology (Kafka -> CNN replicas -> Kafka).",
        epilog=f"subcommands: {', '.join(SUBCOMMANDS)} (python -m gale <subcommand> -h)")
    ap.add_argument("topology_name", metavar="TOPOLOGY_NAME")
    ap.add_argument("input_topic", metavar="INPUT_TOPIC")
    ap.add_argument("output_topic", metavar="OUTPUT_TOPIC")
    ap.add_argument("--config", help="TOML file ([gale] table); CLI > env GALE_* > TOML")
    skip = {"topology_name", "input_topic", "output_topic"}
    for f in fields(GaleConfig):
        if f.name in skip:
            continue
        flag = "--" + f.name.replace("_", "-")
        t = f.type if isinstance(f.type, str) else f.type.__name__
        if t == "bool":
            ap.add_argument(flag, action=argparse.BooleanOptionalAction, default=None)
        else:
            kw = dict(default=None, type={"int": int, "float": float}.get(t, str))
            if f.name in CHOICES:
                kw["choices"] = CHOICES[f.name]
            ap.add_argument(flag, **kw)
    return ap


def parse_topology_args(argv: List[str]) -> GaleConfig:
    ns = vars(_topology_parser().parse_args(argv))
    toml_path = ns.pop("config")
    return from_sources(cli=ns, toml_path=toml_path)


def profile_command(cfg: GaleConfig, argv: List[str]) -> List[str]:
    """The rocprofv3 command that re-runs this topology (minus --profile) with roctx ranges on.

    Kernel dispatches + roctx markers + per-kernel stats land in ``cfg.profile`` (a directory).
    The program runs as a CHILD of this (GPU-untouched) process, right after ``--``: rocprofv3
    initialises the GPU in the profiled process, so no launcher may sit in between.
    """
    rest: List[str] = []
    skip_next = False
    for i, tok in enumerate(argv):
        if skip_next:
            skip_next = False
            continue
        if tok == "--profile":
            skip_next = True
            continue
        if tok.startswith("--profile="):
            continue
        rest.append(tok)
    return ["rocprofv3", "--kernel-trace", "--marker-trace", "--stats", "-d", cfg.profile,
            "-o", cfg.topology_name, "--", sys.executable, "-m", "gale", *rest, "--trace"]


def cmd_run(argv: List[str]) -> int:
    from gale.topology import (AlreadyAliveError, InvalidTopologyError, RankFailedError,
                               run_topology)

    cfg = parse_topology_args(argv)
    if cfg.ranks > 0 and not os.environ.get("GALE_SUPERVISED"):
        # the supervisor: one child process per rank, respawned when it dies (never touches
        # a GPU itself; gale/supervisor.py)
        from gale.supervisor import run_supervised

        logging.basicConfig(level=getattr(logging, cfg.log_level.upper(), logging.INFO),
                            format="%(asctime)s %(name)s %(levelname)s %(message)s")
        return run_supervised(cfg, argv)
    if cfg.profile:
        import subprocess

        # one HW queue per HIP stream in the profiled child: rocprofv3's queue interception
        # crashed when several of the engine's streams shared a HW queue and submitted
        # concurrently (GPU_MAX_HW_QUEUES=4 default; profiles/archive/r3_e2e_kernel_stats_default.csv)
        env = dict(os.environ)
        env.setdefault("GPU_MAX_HW_QUEUES", "32")
        return subprocess.call(profile_command(cfg, argv), env=env)
    logging.basicConfig(level=getattr(logging, cfg.log_level.upper(), logging.INFO),
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    try:
        final = run_topology(cfg)
    except AlreadyAliveError as e:  # MainTopology.java:79-80 logs and returns
        logging.getLogger("gale").error("%s", e)
        return 1
    except InvalidTopologyError as e:
        logging.getLogger("gale").error("invalid topology: %s", e)
        return 2
    except RankFailedError as e:  # replaced by the rank supervisor (--ranks)
        logging.getLogger("gale").error("%s", e)
        return 3
    print(json.dumps({k: v for k, v in final.items() if k != "final"}), file=sys.stderr)
    return 0


def cmd_kill(argv: List[str]) -> int:
    from gale.topology import NotAliveError, Registry

    ap = argparse.ArgumentParser(prog="python -m gale kill")
    ap.add_argument("name")
    ap.add_argument("--wait-secs", type=float, default=0.0)
    ap.add_argument("--registry-dir", default=GaleConfig().registry_dir)
    a = ap.parse_args(argv)
    try:
        Registry(a.registry_dir).kill(a.name, a.wait_secs)
    except NotAliveError as e:  # MainTopology.java:85-86
        print(str(e), file=sys.stderr)
        return 1
    return 0


def cmd_list(argv: List[str]) -> int:
    from gale.topology import Registry

    ap = argparse.ArgumentParser(prog="python -m gale list")
    ap.add_argument("--registry-dir", default=GaleConfig().registry_dir)
    a = ap.parse_args(argv)
    for rec in Registry(a.registry_dir).list():
        print(json.dumps(rec))
    return 0


def cmd_broker(argv: List[str]) -> int:
    from gale._native import native

    ap = argparse.ArgumentParser(prog="python -m gale broker")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9092)
    ap.add_argument("--partitions", type=int, default=1)
    ap.add_argument("--topics", default="", help="comma-separated topics to pre-create")
    ap.add_argument("--max-message-bytes", type=int, default=256 << 20)
    ap.add_argument("--duration", type=float, default=0, help="seconds (0 = until Ctrl-C)")
    a = ap.parse_args(argv)
    b = native().kafka.Broker(host=a.host, port=a.port, default_partitions=a.partitions,
                              max_message_bytes=a.max_message_bytes)
    b.start()
    for t in filter(None, a.topics.split(",")):
        b.create_topic(t, a.partitions)
    print(json.dumps({"broker": f"{a.host}:{b.port}", "partitions": a.partitions}), flush=True)
    try:
        t0 = time.time()
        while a.duration <= 0 or time.time() - t0 < a.duration:
            time.sleep(0.5)
    except KeyboardInterrupt:
        pass
    finally:
        b.stop()
    return 0


def cmd_produce(argv: List[str]) -> int:
    from gale._native import native
    from gale.data import encode_records, synthetic_images
    from gale.models import get_model

    ap = argparse.ArgumentParser(prog="python -m gale produce")
    ap.add_argument("topic")
    ap.add_argument("--bootstrap", default="127.0.0.1:9092")
    ap.add_argument("--images", type=int, default=1000)
    ap.add_argument("--images-per-record", type=int, default=1)
    ap.add_argument("--model", default="resnet20", choices=CHOICES["model"])
    ap.add_argument("--rate", type=float, default=0, help="records/s (0 = as fast as possible)")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    net = get_model(a.model)
    recs = encode_records(synthetic_images(a.images, net.input_shape, a.seed),
                          a.images_per_record)
    p = native().kafka.Producer(a.bootstrap, linger_ms=5, batch_size=1 << 20)
    t0 = time.time()
    for i, r in enumerate(recs):
        if a.rate > 0:
            delay = t0 + i / a.rate - time.time()
            if delay > 0:
                time.sleep(delay)
        p.send(a.topic, r)
    p.flush()
    print(json.dumps({"produced": len(recs), "seconds": round(time.time() - t0, 3),
                      **p.stats()}))
    p.close()
    return 0


def cmd_consume(argv: List[str]) -> int:
    from gale._native import native

    ap = argparse.ArgumentParser(prog="python -m gale consume")
    ap.add_argument("topic")
    ap.add_argument("--bootstrap", default="127.0.0.1:9092")
    ap.add_argument("--max", type=int, default=10)
    ap.add_argument("--from-beginning", action="store_true")
    ap.add_argument("--timeout", type=float, default=10.0)
    a = ap.parse_args(argv)
    c = native().kafka.Consumer(a.bootstrap, max_wait_ms=200)
    c.assign(a.topic, [])
    c.seek_to("earliest" if a.from_beginning else "latest")
    n = 0
    t0 = time.time()
    while n < a.max and time.time() - t0 < a.timeout:
        for r in c.poll():
            v = r["value"]
            print(json.dumps({"partition": r["partition"], "offset": r["offset"],
                              "value": None if v is None else v.decode("utf-8", "replace")}))
            n += 1
            if n >= a.max:
                break
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv and argv[0] in SUBCOMMANDS:
        return {"kill": cmd_kill, "list": cmd_list, "broker": cmd_broker,
                "produce": cmd_produce, "consume": cmd_consume}[argv[0]](argv[1:])
    return cmd_run(argv)
