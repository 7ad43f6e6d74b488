#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per kernel (counter_collection.csv)."""
import collections
import csv
import sys


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(sys.argv[1]) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "?")[:60]
            acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for name, ctrs in acc.items():
        print(name)
        for c, vals in sorted(ctrs.items()):
            # one row per (dispatch, counter) after rocprofv3 aggregation: average over dispatches
            print(f"  {c:28s} {sum(vals) / len(vals):16.1f}  (n={len(vals)})")


if __name__ == "__main__":
    main()
