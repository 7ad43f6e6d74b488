#!/usr/bin/env python3
"""DRAM sensitivity of the headline bench: does the per-rank throughput hold
when the other ranks of a socket load the same memory controllers?

profiles/r5_host_budget.txt §4 projects N = 8 from one rank's CPU slice and assumes the socket's
DRAM keeps up with four ranks (~0.55 TB/s of ~0.61 TB/s peak). This tool tests that assumption
on the one-GPU box: bench.py runs next to tools/bin/dram_antagonist, pinned to the GPU's NUMA
node, at several levels of extra DRAM traffic ("stream": T threads of read + non-temporal-write
copies, one core each) and - the control - the same T threads burning CPU with no memory traffic
("burn"). Both take T cores of the job's CPU quota, so the difference between a stream level and
the burn level with the same T is what the DRAM traffic alone costs.

Runs are interleaved (every level once per round, --rounds rounds) and each is one JSON line:
{"mode", "threads", "round", "img_s", "p50_ms", "p99_ms", "antagonist_gbs", ...}.

    python tools/dram_sensitivity.py --levels 0,2,4,6 --rounds 3 --out profiles/x.jsonl
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ANTAGONIST = os.path.join(ROOT, "tools", "bin", "dram_antagonist")


def gpu_node_cpus() -> str:
    """The GPU's NUMA node CPU list, found in a child (this process never initialises HIP)."""
    code = ("from gale.utils import gpu_numa_node, node_cpus\n"
            "print(','.join(map(str, sorted(node_cpus(gpu_numa_node(0))))) or '-')")
    try:
        p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True,
                           text=True, timeout=300)
        last = p.stdout.strip().splitlines()[-1] if p.returncode == 0 and p.stdout.strip() else ""
        return "" if last == "-" else last
    except (subprocess.TimeoutExpired, IndexError):
        return ""


def last_json(text: str):
    for line in reversed(text.splitlines()):
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return None


def run_level(mode: str, threads: int, rnd: int, a, cpus: str, tmp: str) -> dict:
    rep = os.path.join(tmp, f"ant_{mode}_{threads}_{rnd}.jsonl")
    ant = None
    if threads > 0:
        ant = subprocess.Popen([ANTAGONIST, "--mode", mode, "--threads", str(threads),
                                "--seconds", str(a.bench_timeout + 30), "--cpus", cpus,
                                "--buffer-mb", str(a.buffer_mb), "--report", rep])
        time.sleep(2.0)  # buffers touched, streams at speed
    t0 = time.time()
    try:
        p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *a.bench_args],
                           cwd=ROOT, capture_output=True, text=True, timeout=a.bench_timeout)
        r = last_json(p.stdout)
        err = "" if r else (p.stderr or p.stdout)[-1500:]
    except subprocess.TimeoutExpired:
        r, err = None, f"bench timed out after {a.bench_timeout} s"
    t1 = time.time()
    gbs = []
    if ant is not None:
        ant.terminate()
        try:
            ant.wait(10)
        except subprocess.TimeoutExpired:
            ant.kill()
            ant.wait()
        with open(rep) as f:
            rows = [json.loads(x) for x in f if x.strip()]
        # the antagonist's rate while bench.py ran (its first row is the warm-up second)
        gbs = [x["gbs"] for x in rows[1:] if x["t"] >= 2.0 and x["t"] <= 2.0 + (t1 - t0)]
    row = {"mode": mode if threads else "none", "threads": threads, "round": rnd,
           "antagonist_gbs": round(sum(gbs) / len(gbs), 1) if gbs else 0.0,
           "antagonist_cpus": cpus if threads else ""}
    if r is None:
        row["error"] = err
        return row
    row.update({"img_s": r["value"], "p50_ms": r.get("p50_latency_ms"),
                "p99_ms": r.get("p99_latency_ms"), "p999_ms": r.get("p999_latency_ms"),
                "cpu_cores_busy": r.get("cpu_cores_busy_rank0"),
                "cores_by_stage": r.get("cpu_cores_by_stage_rank0"),
                "throttled_ms": (r.get("timed_cgroup_rank0") or {}).get("throttled_ms")})
    return row


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--levels", default="0,2,4,6",
                    help="antagonist thread counts; each > 0 runs as stream AND burn")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--buffer-mb", type=int, default=512)
    ap.add_argument("--bench-timeout", type=int, default=150)
    ap.add_argument("--out", default="")
    ap.add_argument("--tmp", default="/tmp")
    ap.add_argument("bench_args", nargs=argparse.REMAINDER, help="-- bench.py arguments")
    a = ap.parse_args(argv)
    a.bench_args = a.bench_args[1:] if a.bench_args[:1] == ["--"] else a.bench_args
    if not os.path.exists(ANTAGONIST):
        print("build it first: make antagonist", file=sys.stderr)
        return 2
    cpus = gpu_node_cpus()
    levels = [int(x) for x in a.levels.split(",") if x.strip()]
    plan = []
    for t in levels:
        plan += [("none", 0)] if t == 0 else [("stream", t), ("burn", t)]
    out = open(a.out, "a") if a.out else None
    rc = 0
    for rnd in range(a.rounds):
        for mode, t in plan:
            row = run_level(mode, t, rnd, a, cpus, a.tmp)
            line = json.dumps(row)
            print(line, flush=True)
            if out:
                out.write(line + "\n")
                out.flush()
            if "error" in row:
                rc = 1
                break
        if rc:
            break
    return rc


if __name__ == "__main__":
    sys.exit(main())
