#!/usr/bin/env python3
"""Latency-SLO sweep (BASELINE config 5: "ResNet-20 with fp8 weights, high-QPS latency-SLO mode").

Runs ``bench.py --rate R`` (an open-loop feeder appends records at R images/s per GPU; the
broker stamps them with LogAppendTime, so ``record_e2e_ms_p99`` is the exact append ->
produce-ack latency) for increasing offered loads, with the engine's SLO controller on
(``--slo-p99-ms``), and reports the highest offered load whose achieved rate keeps up (>= 97 %
of the offer) with p99 <= the SLO: "max QPS at p99 <= X ms". Every run is a child process.

    python tools/slo_sweep.py --slo-ms 5 --rates 200000,400000,600000 [-- extra bench.py args]
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(rate: float, slo: float, dtype: str, extra: list, timeout: float) -> dict:
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--rate", str(int(rate)),
           "--dtype", dtype, "--steps", "10", "--warmup", "2", "--step-images", "32768",
           "--slo-p99-ms", str(slo)] + extra
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    for line in reversed(p.stdout.splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return {"error": f"rc={p.returncode}", "tail": p.stderr[-1500:]}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--slo-ms", type=float, default=5.0)
    ap.add_argument("--rates", default="100000,200000,400000,600000,800000")
    ap.add_argument("--dtypes", default="bf16,fp8")
    ap.add_argument("--timeout", type=float, default=240.0)
    ap.add_argument("extra", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    extra = a.extra[1:] if a.extra[:1] == ["--"] else a.extra
    summary = {}
    for dtype in a.dtypes.split(","):
        best = None
        for rate in [float(x) for x in a.rates.split(",")]:
            r = run(rate, a.slo_ms, dtype, extra, a.timeout)
            if "error" in r:
                print(json.dumps({"dtype": dtype, "rate": rate, **r}), flush=True)
                break
            p99 = r["record_e2e_ms_p99"]
            ok = r["value"] >= 0.97 * rate and p99 <= a.slo_ms
            print(json.dumps({"dtype": dtype, "offered": rate, "achieved": r["value"],
                              "record_e2e_ms_p50": r["record_e2e_ms_p50"],
                              "record_e2e_ms_p99": p99, "p99_fetch_to_ack_ms":
                                  r["p99_latency_ms"], "batch_images_mean":
                                  r["batch_images_mean"], "meets_slo": ok}), flush=True)
            if ok:
                best = rate
        summary[dtype] = best
    print(json.dumps({"slo_p99_ms": a.slo_ms, "max_offered_images_per_s_meeting_slo": summary}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
