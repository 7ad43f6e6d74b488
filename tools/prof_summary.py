#!/usr/bin/env python3
"""Summarise a rocprofv3 run_results.db (kernel + memory-copy stats) as CSV-ish text.

usage: python tools/prof_summary.py gpurun_out/prof/run_results.db [--top 25]
"""
import argparse
import sqlite3


def busy(c, top, tail_s=0.0):
    ev = []
    lo = 0
    if tail_s > 0:
        lo = c.execute("select max(end) from kernels").fetchone()[0] - int(tail_s * 1e9)
    for name, st, en in c.execute("select name, start, end from kernels where end > start "
                                  "and start >= ?", (lo,)):
        ev.append((st, 1, name))
        ev.append((en, -1, name))
    if not ev:
        print("no kernels")
        return
    ev.sort(key=lambda e: (e[0], e[1]))
    active = {}
    share = {}
    busy_ns = 0
    t_prev = ev[0][0]
    for t, d, name in ev:
        k = sum(active.values())
        if k and t > t_prev:
            seg = t - t_prev
            busy_ns += seg
            for n, m in active.items():
                share[n] = share.get(n, 0.0) + seg * m / k
        t_prev = t
        active[name] = active.get(name, 0) + d
        if active[name] == 0:
            del active[name]
    span = ev[-1][0] - ev[0][0]
    print(f"span_ms,{span / 1e6:.1f},busy_ms,{busy_ns / 1e6:.1f},busy_pct,{100 * busy_ns / span:.1f}")
    print("kernel,attributed_us,pct_of_busy")
    for name, v in sorted(share.items(), key=lambda kv: -kv[1])[:top]:
        short = name if len(name) < 110 else name[:107] + "..."
        print(f'"{short}",{v / 1e3:.1f},{100 * v / busy_ns:.1f}')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--by-grid", action="store_true",
                    help="one row per (kernel, grid size): per-layer view of a plan")
    ap.add_argument("--busy", action="store_true",
                    help="GPU busy share of the traced span, and each kernel's share of the "
                         "busy time with concurrent kernels splitting a time slice evenly (the "
                         "per-kernel durations double-count overlap when streams run together)")
    ap.add_argument("--tail-s", type=float, default=0.0,
                    help="with --busy: only the kernels of the trace's last S seconds (the timed "
                         "window of a bench run, without its start-up)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    if a.busy:
        busy(c, a.top, a.tail_s)
        return
    key = "name || ' grid=' || grid_x || 'x' || grid_y" if a.by_grid else "name"
    rows = c.execute(
        f"select {key}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
        "from kernels group by 1 order by sum(end-start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    print("kernel,calls,total_us,avg_us,min_us,max_us,pct")
    for name, n, tot, avg, mn, mx in rows[:a.top]:
        if a.by_grid and " grid=" in name:
            base, grid = name.rsplit(" grid=", 1)
            name = (base if len(base) < 70 else base[:67] + "...") + " grid=" + grid
        short = name if len(name) < 110 else name[:107] + "..."
        print(f'"{short}",{n},{tot/1e3:.1f},{avg/1e3:.2f},{mn/1e3:.2f},{mx/1e3:.2f},'
              f"{100*tot/total:.1f}")
    try:
        rg = c.execute(
            "select json_extract(extdata, '$.message'), count(*), sum(end-start), avg(end-start), "
            "count(distinct tid) from regions where extdata like '%message%' group by 1 "
            "order by 3 desc").fetchall()
    except sqlite3.Error:
        rg = []
    if rg:
        print("\nroctx_range,calls,total_us,avg_us,threads")
        for name, n, tot, avg, nt in rg:
            print(f"{name},{n},{tot/1e3:.1f},{avg/1e3:.2f},{nt}")
    try:
        mc = c.execute("select src_agent_type||'->'||dst_agent_type, count(*), sum(end-start), "
                       "sum(size) from memory_copies group by 1").fetchall()
    except sqlite3.Error:
        mc = []
    if mc:
        print("\ncopy,calls,total_us,bytes,GB_per_s")
        for k, n, tot, sz in mc:
            print(f"{k},{n},{tot/1e3:.1f},{sz},{(sz or 0)/max(tot,1):.2f}")


if __name__ == "__main__":
    main()
