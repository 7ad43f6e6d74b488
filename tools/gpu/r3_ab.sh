#!/bin/bash
# A/B of bench.py variants with a 100 ms timeline each: tools/gpu/r3_ab.sh OUTDIR "name|args" ...
set -o pipefail
out=$1; shift
mkdir -p "$out"
for spec in "$@"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 $args --timeline "$out/tl_$name.jsonl" \
    > "$out/b_$name.json" 2> "$out/b_$name.err" || exit $?
done
