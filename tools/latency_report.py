#!/usr/bin/env python3
"""Place a latency tail in time: per window of the latency phase, the record latency quantiles
and each stage's p99 (from ``bench.py --latency-dump``), next to what the host did in that
window (from ``bench.py --timeline``: completion rate, cgroup cores and throttling, queue).

    python tools/latency_report.py gpurun_out/lat/lat.npz [gpurun_out/lat/tl.jsonl] [--ms 100]
"""

from __future__ import annotations

import argparse
import json

import numpy as np

STAGES = ("broker_source", "queue", "replica", "sink")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("npz")
    ap.add_argument("timeline", nargs="?")
    ap.add_argument("--ms", type=float, default=100.0)
    a = ap.parse_args(argv)
    z = np.load(a.npz)
    lat, t = z["latency_us"].astype(np.float64), z["ack_t_ns"] / 1e9
    st = {k: z[k].astype(np.float64) for k in STAGES if k in z}
    tl = []
    if a.timeline:
        tl = [json.loads(x) for x in open(a.timeline) if x.strip()]
        tl = [r for r in tl if r.get("phase") == "latency" and "mono" in r]
    w = a.ms / 1e3
    t0 = t.min()
    nb = int((t.max() - t0) / w) + 1
    b = ((t - t0) / w).astype(int)
    print(f"{'t_s':>5} {'n':>7} {'p50':>6} {'p99':>6} {'max':>6} | stage p99 (ms): "
          + " ".join(f"{k[:8]:>8}" for k in st) + " | host")
    for i in range(nb):
        sel = b == i
        if not sel.any():
            continue
        row = (f"{i * w:5.2f} {int(sel.sum()):7d} {np.percentile(lat[sel], 50) / 1e3:6.2f} "
               f"{np.percentile(lat[sel], 99) / 1e3:6.2f} {lat[sel].max() / 1e3:6.2f} |"
               + "".join(f" {np.percentile(v[sel], 99) / 1e3:8.2f}" for v in st.values()) + " |")
        if tl:
            mid = t0 + (i + 0.5) * w
            r = min(tl, key=lambda x: abs(x["mono"] - w / 2 - mid))
            row += (f" rate={r.get('rate')} cg={r.get('cg_cores')} thr={r.get('throttled_ms')}"
                    f" q={r.get('queue')} busy={r.get('busy')}")
        print(row)
    print("whole window: p50 %.3f p99 %.3f p99.9 %.3f ms; stage p50/p99: %s" % (
        np.percentile(lat, 50) / 1e3, np.percentile(lat, 99) / 1e3, np.percentile(lat, 99.9) / 1e3,
        {k: (round(np.percentile(v, 50) / 1e3, 3), round(np.percentile(v, 99) / 1e3, 3))
         for k, v in st.items()}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
