#!/usr/bin/env python3
"""Per-kernel time summary of a rocprofv3 SQLite database (rocprofv3 --kernel-trace writes
<out>_results.db): name, dispatches, total / mean / p50 microseconds and share of the summed
kernel time, plus the span of the trace. Text out, to commit under profiles/.

    python tools/rocpd_summary.py gpurun_out/x/prof/run_results.db > profiles/x.txt
"""

import sqlite3
import sys

import numpy as np


def main(path: str) -> int:
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, start, end from kernels"))
    if not rows:
        print("no kernel dispatches")
        return 1
    by = {}
    for name, s, e in rows:
        by.setdefault(name, []).append(e - s)
    t0 = min(r[1] for r in rows)
    t1 = max(r[2] for r in rows)
    total = sum(sum(v) for v in by.values())
    print(f"# {path}: {len(rows)} dispatches over {(t1 - t0) / 1e9:.3f} s of trace; "
          f"summed kernel time {total / 1e9:.3f} s")
    print(f"{'kernel':72s} {'n':>8s} {'total ms':>10s} {'mean us':>8s} {'p50 us':>8s} {'share':>6s}")
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        a = np.asarray(v, dtype=np.float64)
        short = name if len(name) <= 72 else name[:69] + "..."
        print(f"{short:72s} {len(a):8d} {a.sum() / 1e6:10.1f} {a.mean() / 1e3:8.1f} "
              f"{np.median(a) / 1e3:8.1f} {100 * a.sum() / total:5.1f}%")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
