#!/bin/bash
# Config 2 headline vs socket buffer size (GALE_SOCK_BUF; default 8 MiB): does less data in
# flight per connection keep the receive copy's source in cache?
set -o pipefail
d=gpurun_out/sockbuf
mkdir -p $d
: > $d/ab.jsonl
sysctl net.core.rmem_max net.core.wmem_max net.ipv4.tcp_rmem 2>/dev/null | tee $d/sysctl.txt
for r in 1 2; do
  for b in 8388608 2097152 1048576; do
    GALE_SOCK_BUF=$b timeout -k 10 240 python bench.py > $d/b.json 2> $d/b.err \
        || { tail -5 $d/b.err; exit 1; }
    tail -1 $d/b.json | sed "s/^{/{\"sock_buf\": $b, /" >> $d/ab.jsonl
    tail -1 $d/b.json | cut -c1-110
  done
done
