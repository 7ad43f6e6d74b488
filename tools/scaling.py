#!/usr/bin/env python3
"""Scaling curve of the headline benchmark (BASELINE.json: whole-node images/s + p50 latency,
CIFAR-10 ResNet-20 at 1/2/4/8 GPUs).

Runs ``bench.py --gpus N`` once per GPU count N on ONE node, exactly as the round driver does:
a plain process, which for N > 1 starts ``torch.distributed.run`` itself (one rank per GPU, RCCL
over xGMI, rendezvous on 127.0.0.1; bench.py ``launch_ranks``) -- and
prints one JSON line per N plus a summary with the per-N images/s, p50/p99 latency and the
weak-scaling efficiency value(N) / (N * value(1)). Every run is a child process (never an exec),
bounded by ``--timeout``; the sweep stops at the first failing N.

Placement (``--placements floating,slices``, the default): at every N > 1 the sweep runs both
host placements of the ranks - "floating" (each rank's threads float over its GPU's whole NUMA
node, bench.py's default) and "slices" (``--rank-slices``: each rank owns a disjoint slice of
whole cores of that node) - back to back, and reports each with per-rank img/s and busy cores.
The summary's ``placement`` block names the faster placement at the largest N and by how much:
the first 8-GPU run decides the default by itself.

The reference has no benchmark of its own (E12 storm-perf is declared in
pom.xml:44-54 but unused); this is the new framework's storm-perf-style scaling driver.

    python tools/scaling.py --gpus 1,2,4,8 --steps 100 --warmup 10 [-- extra bench.py args]
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


PLACEMENT_FLAGS = {"floating": [], "slices": ["--rank-slices"]}


def plan(counts: list, placements: list) -> list:
    """(N, placement) runs in order: N = 1 has one placement (a single rank), every N > 1 runs
    each requested placement back to back."""
    out = []
    for n in counts:
        for pl in (placements[:1] if n == 1 else placements):
            out.append((n, pl))
    return out


def bench_cmd(n: int, steps: int, warmup: int, extra: list, stub: bool = False,
              single_process: bool = False, placement: str = "floating") -> list:
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", str(steps),
            "--warmup", str(warmup)] + (["--stub"] if stub else []) + list(extra)
    if n > 1 and not single_process:
        args += PLACEMENT_FLAGS[placement]
    # n > 1 per-process: bench.py launches its own ranks (the driver's entry point)
    return [sys.executable] + args + (["--single-process"] if single_process else [])


def last_json(text: str):
    for line in reversed(text.splitlines()):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return None


def efficiency(results: dict) -> dict:
    """Weak-scaling efficiency value(N) / (N * value(1)) for every measured N."""
    if 1 not in results:
        return {}
    base = results[1]["value"]
    return {n: round(r["value"] / (n * base), 4) for n, r in sorted(results.items())}


def per_rank(r: dict) -> list:
    """Each rank's img/s, busy cores and CPU slice from a bench.py JSON line."""
    return [{"rank": x.get("rank"), "img_s": x.get("img_s"), "cores": x.get("cores"),
             "cpus": x.get("cpus")} for x in (r.get("ranks") or [])]


def placement_verdict(by_pl: dict, margin: float = 0.02) -> dict:
    """by_pl: placement -> {N: result}. At the largest N measured under every placement, the
    faster one; "floating" (the default) is kept unless another beats it by > margin."""
    common = set.intersection(*(set(k for k in v if k > 1) for v in by_pl.values())) \
        if by_pl else set()
    if len(by_pl) < 2 or not common:
        return {}
    n = max(common)
    vals = {pl: by_pl[pl][n]["value"] for pl in by_pl}
    best = max(vals, key=vals.get)
    base = vals.get("floating", vals[best])
    gain = vals[best] / base - 1 if base else 0.0
    choice = best if best != "floating" and gain > margin else "floating"
    return {"n_gpus": n, "images_per_s": vals, "faster": best,
            "gain_over_floating": round(gain, 4), "default": choice,
            "rule": f"--rank-slices becomes the default only if it beats floating by > "
                    f"{margin:.0%} at the largest N"}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--gpus", default="1,2,4,8", help="comma-separated GPU counts")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--stub", action="store_true", help="CPU stub replicas (gloo; plumbing)")
    ap.add_argument("--timeout", type=float, default=900.0, help="seconds per bench run")
    ap.add_argument("--out", default="", help="also append the JSON lines to this file")
    ap.add_argument("--mode", default="per-process",
                    choices=["per-process", "single-process", "both"],
                    help="per-process: one torch.distributed rank per GPU; single-process: one "
                         "engine driving every GPU (bench.py --single-process)")
    ap.add_argument("--placements", default="floating,slices",
                    help="host placements to run at every N > 1 (comma list of floating, "
                         "slices; N = 1 runs the first)")
    ap.add_argument("--dry-run", action="store_true",
                    help="print, per N, the command and per-rank configuration the sweep would "
                         "run (bench.py --print-config), without running anything")
    ap.add_argument("extra", nargs=argparse.REMAINDER, help="-- extra bench.py arguments")
    a = ap.parse_args(argv)
    extra = a.extra[1:] if a.extra[:1] == ["--"] else a.extra
    counts = [int(x) for x in a.gpus.split(",") if x.strip()]
    a.placement_list = [x.strip() for x in a.placements.split(",") if x.strip()]
    for pl in a.placement_list:
        if pl not in PLACEMENT_FLAGS:
            ap.error(f"unknown placement {pl!r} (floating, slices)")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MASTER_ADDR="127.0.0.1")
    modes = ["per-process", "single-process"] if a.mode == "both" else [a.mode]
    rc = 0
    for mode in modes:
        rc |= (dry_run if a.dry_run else sweep)(a, counts, extra, env, mode)
    return rc


def _pin_from(cfg: dict, extra: list) -> list:
    """The N = 1 run's per-GPU sizing as bench.py flags, pinned for every larger N."""
    pinned = []
    for flag, key in (("--partitions", "partitions_per_gpu"),
                      ("--replicas-per-gpu", "replicas_per_gpu"),
                      ("--decode-threads", "decode_threads"), ("--batch", "max_batch"),
                      ("--step-images", "step_images_per_gpu")):
        if cfg.get(key) and flag not in extra:
            pinned += [flag, str(cfg[key])]
    return pinned


def dry_run(a, counts, extra, env, mode) -> int:
    """--dry-run: one line per (N, placement) with the exact bench.py command and its per-rank
    config (CPU slices included)."""
    pinned: list = []
    placements = a.placement_list if mode == "per-process" else ["floating"]
    for n, pl in plan(counts, placements):
        cmd = bench_cmd(n, a.steps, a.warmup, extra + pinned, a.stub,
                        single_process=mode == "single-process", placement=pl)
        p = subprocess.run(cmd + ["--print-config"], cwd=ROOT, env=env, capture_output=True,
                           text=True, timeout=300)
        cfg = None
        for line in p.stdout.splitlines():
            if line.startswith("{"):
                cfg = json.loads(line)
        if p.returncode != 0 or cfg is None:
            print(json.dumps({"n_gpus": n, "error": f"rc={p.returncode}",
                              "tail": p.stderr[-2000:]}))
            return 1
        if not pinned:
            pinned = _pin_from(cfg, extra)
        print(json.dumps({"mode": mode, "n_gpus": n, "placement": pl, "cmd": " ".join(cmd[1:]),
                          "config": cfg}), flush=True)
    return 0


def sweep(a, counts, extra, env, mode) -> int:
    by_pl: dict = {}
    pinned: list = []
    placements = a.placement_list if mode == "per-process" else ["floating"]
    runs = plan(counts, placements)
    done = 0
    for n, pl in runs:
        # weak scaling compares equal per-GPU work: every N > first runs with the per-GPU
        # configuration the first run chose for itself (bench.py sizes replicas per GPU from the
        # rank's CPU share, which shrinks as more ranks share the node's CPUs)
        cmd = bench_cmd(n, a.steps, a.warmup, extra + pinned, a.stub,
                        single_process=mode == "single-process", placement=pl)
        try:
            p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True,
                               timeout=a.timeout)
        except subprocess.TimeoutExpired:
            print(json.dumps({"n_gpus": n, "placement": pl,
                              "error": f"timed out after {a.timeout:.0f}s"}))
            break
        r = last_json(p.stdout)
        if p.returncode != 0 or r is None:
            tail = (p.stderr or p.stdout)[-2000:]
            print(json.dumps({"n_gpus": n, "placement": pl, "error": f"rc={p.returncode}",
                              "tail": tail}))
            break
        done += 1
        by_pl.setdefault(pl, {})[n] = r
        if n == 1:  # the single-rank result is every placement's N = 1 point
            for other in placements:
                by_pl.setdefault(other, {})[1] = r
        if not pinned:
            cfg = r.get("config", {})
            per_gpu_parts = cfg.get("partitions", 0) // max(1, r.get("n_gpus", 1))
            if per_gpu_parts and "--partitions" not in extra:
                pinned += ["--partitions", str(per_gpu_parts)]
            for flag, key in (("--replicas-per-gpu", "replicas_per_gpu"),
                              ("--decode-threads", "decode_threads"),
                              ("--batch", "max_batch"),
                              ("--step-images", "step_images_per_gpu")):
                if key in cfg and flag not in extra:
                    pinned += [flag, str(cfg[key])]
        row = dict(r, placement=pl, per_rank=per_rank(r))
        print(json.dumps(row), flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(json.dumps(row) + "\n")
    summary = {"mode": mode, "scaling": {}}
    for pl, results in by_pl.items():
        eff = efficiency(results)
        summary["scaling"][pl] = {
            str(n): {"images_per_s": r["value"], "p50_ms": r.get("p50_latency_ms"),
                     "p99_ms": r.get("p99_latency_ms"), "efficiency": eff.get(n),
                     "replicas_per_gpu": r["config"].get("replicas_per_gpu"),
                     "global_batch": r["config"].get("global_batch"),
                     "cpu_cores_busy_rank0": r.get("cpu_cores_busy_rank0"),
                     "per_rank": per_rank(r)}
            for n, r in sorted(results.items())}
    summary["placement"] = placement_verdict(by_pl)
    print(json.dumps(summary), flush=True)
    return 0 if done == len(runs) else 1


if __name__ == "__main__":
    sys.exit(main())
