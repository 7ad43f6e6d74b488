#!/bin/bash
# latency tail A/B: socket buffers (explicit 8 MiB request, clamped by wmem_max, vs kernel
# autotuning) with three 0.8-load latency phases per run; then the SLO sweep without the
# engine's SLO controller
set -o pipefail
d=gpurun_out/tailab
mkdir -p $d
export TMPDIR=/tmp
cat /proc/sys/net/core/wmem_max /proc/sys/net/core/rmem_max /proc/sys/net/ipv4/tcp_wmem /proc/sys/net/ipv4/tcp_rmem > $d/sysctl.txt 2>&1
for i in 1 2; do
  for v in default 0; do
    if [ $v = default ]; then unset GALE_SOCK_BUF; else export GALE_SOCK_BUF=$v; fi
    timeout -k 10 300 python bench.py --latency-sweep 0.8 --latency-repeat 2 > $d/b_${v}_$i.log 2>&1 || { tail -20 $d/b_${v}_$i.log; exit 1; }
    grep '^{' $d/b_${v}_$i.log | tail -1 > $d/b_${v}_$i.json
    python3 -c "
import json; d=json.load(open('$d/b_${v}_$i.json'))
print('$v', $i, d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['latency_stages_ms']['broker_source'], [(x['p99_ms'], x['stages_ms']['broker_source'][1]) for x in d.get('latency_sweep', [])], d['cpu_cores_by_stage_rank0'])"
  done
done
unset GALE_SOCK_BUF
timeout -k 10 600 python tools/slo_sweep.py --slo-ms 5 --repeat 2 --no-controller --loads 0.6,0.7,0.8,0.9,0.95 > $d/slo_nc.jsonl 2> $d/slo_nc.err || { tail -20 $d/slo_nc.err; exit 1; }
tail -1 $d/slo_nc.jsonl
