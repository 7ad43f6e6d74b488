#!/bin/bash
# per-layer kernel times of the ResNet-50 forward at batch 256 (rocprofv3 kernel trace, one row per
# kernel and grid size)
set -o pipefail
d=gpurun_out/fwdprof
mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d $d/prof -o run -- \
    python tools/bench_forward.py --model resnet50 --batches 256 --iters 20 > $d/fwd.log 2>&1 || exit 1
db=$(find $d/prof -name '*.db' | head -1)
python tools/prof_summary.py $db --by-grid --top 60 > $d/by_grid.txt
python - $db > $d/layers.txt <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, grid_x, start, end from kernels order by start").fetchall()
# the last 20 forwards: find the period from the stem_pack kernel
idx = [i for i, r in enumerate(rows) if 'stem_pack' in r[0]]
per = idx[-1] - idx[-2]
tail = rows[idx[-6]:idx[-1]]  # 5 forwards
n = per
acc = {}
for k in range(5):
    for j in range(n):
        nm, g, s, e = tail[k * n + j]
        key = (j, nm.split('(')[0][-60:], g)
        acc[key] = acc.get(key, 0) + (e - s) / 5
tot = 0
for (j, nm, g), us in sorted(acc.items()):
    tot += us
    print(f"{j:3d} {us/1e3:8.1f} us  grid={g:<8d} {nm}")
print("total_us", round(tot / 1e3, 1))
PY
tail -70 $d/layers.txt
rm -rf $d/prof
