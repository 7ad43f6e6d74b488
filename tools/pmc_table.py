#!/usr/bin/env python3
"""Per-kernel PMC + timing table (roofline evidence) from rocprofv3 CSV outputs.

    python tools/pmc_table.py --trace kernel_trace.csv --pmc pass1.csv pass2.csv ... [--peak-tf 2500]

Groups dispatches by (kernel, grid size) - one group per layer shape - averages every counter
over the group's dispatches and prints, per group: mean duration, MFMA FLOPs (512 FLOPs per
SQ_INSTS_VALU_MFMA_MOPS_* unit, the Omniperf convention), achieved TFLOP/s and % of the dense
peak, HBM bytes (FETCH_SIZE + WRITE_SIZE, KB units) and TB/s, MFMA-busy fraction, LDS bank
conflicts per LDS instruction, waves and L2 hit rate.
"""

import argparse
import collections
import csv


def key(row):
    name = row.get("Kernel_Name", "?").replace("(anonymous namespace)::", "")
    short = name.replace("void ", "").replace("gale::", "").split("(")[0]
    grid = row.get("Grid_Size") or row.get("Grid_Size_X") or "?"
    return f"{short[:58]} grid={grid}"


def layer_labels(model: str, batch: int):
    """Plan op labels, analytical FLOPs and minimum HBM bytes per op (dispatch order)."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from gale.models import get_model
    from gale.models.graph import build_plan

    net = get_model(model)
    ops, _ = build_plan(net, 0, "bf16", fused=True)
    out = []
    for op in ops:
        if op["kind"] == 0:
            L = net.layers[op["layer"]]
            d = op["conv"]
            m = batch * d["Ho"] * d["Wo"]
            fl = 2.0 * m * d["Cout"] * d["K"]
            by = 2.0 * (batch * d["H"] * d["W"] * d["Cin"] + m * d["Cout"] * (2 if d.get("has_res")
                                                                               else 1))
            by += d["Npad"] * d["Kpad"] * 2
            out.append((f"{L.name} {d['KH']}x{d['KW']}/{d['stride']} {d['Cin']}->{d['Cout']} "
                        f"@{d['Ho']}x{d['Wo']}", fl, by))
        elif op["kind"] == 9:  # OP_BOTTLENECK: a whole 56x56 block (bottleneck_fused.hip)
            cin, down = op["p"][0], op["p"][1]
            blk = net.layers[op["layer"]].name.rsplit(".", 1)[0]
            m = batch * 56 * 56
            fl = 2.0 * m * (cin * 64 + 576 * 64 + 64 * 256 + (64 * 256 if down else 0))
            by = 2.0 * m * (cin + 256 + (0 if down else 256))
            out.append((f"{blk} fused bottleneck {cin}->256{' +proj' if down else ''}", fl, by))
        elif op["kind"] == 10:  # OP_STEM_POOL: stem conv + max-pool (stem_pool.hip)
            d = op["conv"]
            m = batch * d["Ho"] * d["Wo"]
            fl = 2.0 * m * d["Cout"] * d["K"] * 9 / 8  # (+1 recomputed window row in 8)
            by = 2.0 * (batch * d["H"] * d["W"] * 4 + batch * 56 * 56 * d["Cout"])
            out.append(("stem 7x7/2 + maxpool 3x3/2 (fused) @56x56", fl, by))
        elif op["kind"] == 11:  # OP_CONV_PROJ: conv3 + strided projection (conv2d_gemm_proj)
            d = op["conv"]
            H2, W2, Cin2 = op["p"][:3]
            m = batch * d["Ho"] * d["Wo"]
            fl = 2.0 * m * d["Cout"] * (d["K"] + Cin2)
            by = 2.0 * (batch * d["H"] * d["W"] * d["Cin"] + m * Cin2 + m * d["Cout"])
            by += d["Npad"] * (d["Kpad"] + op["p"][4]) * 2
            blk = net.layers[op["layer"]].name.rsplit(".", 1)[0]
            out.append((f"{blk} conv3 1x1 {d['Cin']}->{d['Cout']} + proj 1x1/2 {Cin2} @"
                        f"{d['Ho']}x{d['Wo']}", fl, by))
        elif op["kind"] == 6:
            out.append(("stem_pack (fp32 -> bf16 [224][230][4])", 0.0, 0.0))
        elif op["kind"] == 2:
            out.append(("avgpool 7x7 (global)", 0.0, 0.0))
        elif op["kind"] == 4:
            out.append(("softmax 1000", 0.0, 0.0))
        else:
            out.append((f"op{op['kind']}", 0.0, 0.0))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--pmc", nargs="+", default=[])
    ap.add_argument("--peak-tf", type=float, default=2500.0, help="dense bf16 peak TFLOP/s")
    ap.add_argument("--peak-tbs", type=float, default=8.0, help="HBM peak TB/s")
    ap.add_argument("--mops", default="SQ_INSTS_VALU_MFMA_MOPS_BF16")
    ap.add_argument("--xcds", type=int, default=8)
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--label-model", default="", help="label dispatches by the model's plan")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--show", default="", help="extra counters (comma list) printed per layer "
                    "as per-CU-cycle rates: value / (GRBM_GUI_ACTIVE / xcds * cus)")
    a = ap.parse_args()
    if a.label_model:
        return per_layer(a)
    dur = collections.defaultdict(list)
    with open(a.trace) as f:
        for row in csv.DictReader(f):
            dur[key(row)].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in a.pmc:
        with open(path) as f:
            for row in csv.DictReader(f):
                ctr[key(row)][row["Counter_Name"]].append(float(row["Counter_Value"]))
    print(f"{'kernel (grid = threads)':70s} {'n':>4s} {'us':>8s} {'TF/s':>7s} {'%pk':>5s} "
          f"{'GB':>7s} {'TB/s':>6s} {'mfma%':>6s} {'ldsCf':>6s} {'L2hit':>6s}")
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        us = sum(dur[k]) / len(dur[k]) / 1e3
        c = {n: sum(v) / len(v) for n, v in ctr.get(k, {}).items()}
        flops = 512.0 * c.get(a.mops, 0.0)
        tf = flops / (us * 1e-6) / 1e12 if us > 0 else 0.0
        gb = (c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024 / 1e9
        tbs = gb / (us * 1e-6) / 1e3 if us > 0 else 0.0
        # MFMA utilisation: busy MFMA cycles over (kernel cycles x CUs x 4 SIMDs); the GUI-active
        # counter is summed over the XCDs
        cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / a.xcds
        mfma = 100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (cyc * a.cus * 4) if cyc else 0.0
        lds = c.get("SQ_INSTS_LDS", 0.0)
        cf = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds if lds else 0.0
        hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        l2 = 100.0 * hit / (hit + miss) if hit + miss else 0.0
        print(f"{k:70s} {len(dur[k]):4d} {us:8.1f} {tf:7.1f} {100 * tf / a.peak_tf:5.1f} "
              f"{gb:7.3f} {tbs:6.2f} {mfma:6.1f} {cf:6.2f} {l2:6.1f}")
    print("\nraw counter means per group:")
    for k in sorted(ctr):
        print(k)
        for n, v in sorted(ctr[k].items()):
            print(f"    {n:34s} {sum(v) / len(v):18.1f}")


def per_layer(a):
    """Dispatches in launch order, labelled with the plan's ops (one eager forward = one op
    sequence); counters joined by dispatch position within the forward."""
    labels = layer_labels(a.label_model, a.batch)
    n = len(labels)
    show = [k for k in a.show.split(",") if k]

    def ordered(path):
        rows = []
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Kernel_Name", "").startswith("__amd"):
                    continue
                rows.append(row)
        return rows

    tr = [r for r in ordered(a.trace)]
    tr.sort(key=lambda r: int(r.get("Dispatch_Id", 0)))
    tr = tr[len(tr) % n:]  # whole forwards only
    dur = collections.defaultdict(list)
    for i, r in enumerate(tr):
        dur[i % n].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in a.pmc:
        rows = ordered(path)
        ids = sorted({int(r.get("Dispatch_Id", 0)) for r in rows})
        ids = ids[len(ids) % n:]
        pos = {d: i % n for i, d in enumerate(ids)}
        for r in rows:
            d = int(r.get("Dispatch_Id", 0))
            if d in pos:
                ctr[pos[d]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"{'layer':44s} {'us':>7s} {'TF/s':>6s} {'%pk':>5s} {'minGB':>6s} {'TB/s':>5s} "
          f"{'hbmGB':>6s} {'mfma%':>6s} {'ldsCf':>6s} {'L2hit':>6s}"
          + "".join(f" {k[3:17] if k.startswith('SQ_') else k[:14]:>14s}" for k in show))
    tot_us = tot_fl = 0.0
    for i in range(n):
        name, fl, by = labels[i]
        us = sum(dur[i]) / max(1, len(dur[i])) / 1e3
        c = {k: sum(v) / len(v) for k, v in ctr[i].items()}
        tot_us += us
        tot_fl += fl
        tf = fl / (us * 1e-6) / 1e12 if us else 0.0
        tbs = by / (us * 1e-6) / 1e12 if us else 0.0
        hbm = (c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024 / 1e9
        cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / a.xcds
        mfma = 100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (cyc * a.cus * 4) if cyc else 0.0
        lds = c.get("SQ_INSTS_LDS", 0.0)
        cf = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds if lds else 0.0
        hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        l2 = 100.0 * hit / (hit + miss) if hit + miss else 0.0
        print(f"{name:44s} {us:7.1f} {tf:6.0f} {100 * tf / a.peak_tf:5.1f} {by / 1e9:6.3f} "
              f"{tbs:5.2f} {hbm:6.3f} {mfma:6.1f} {cf:6.2f} {l2:6.1f}"
              + "".join(f" {c.get(k, 0.0) / (cyc * a.cus) if cyc else 0.0:14.3f}" for k in show))
    print(f"{'TOTAL':44s} {tot_us:7.1f} {tot_fl / (tot_us * 1e-6) / 1e12:6.0f}")


if __name__ == "__main__":
    main()
