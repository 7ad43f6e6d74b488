#!/bin/bash
# ResNet-50 end to end, GPU-bound: text pack vs none, pinned budget, with engine counters, and a
# kernel trace of the timed window's busy share
set -o pipefail
d=gpurun_out/diag4
mkdir -p $d
: > $d/runs.jsonl
for spec in "pack|" "nopack|--no-text-pack" "pack16g|--pinned-fetch-mb 8192" "pack_r3|--replicas-per-gpu 3"; do
  label=${spec%%|*}; args=${spec#*|}
  timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 --all-stats $args \
    > $d/one.jsonl 2> $d/$label.err || { tail -5 $d/$label.err; exit 1; }
  python - "$label" <<'PY'
import json, sys
r = json.loads(open('gpurun_out/diag4/one.jsonl').read().strip().splitlines()[-1])
r['label'] = sys.argv[1]
open('gpurun_out/diag4/runs.jsonl', 'a').write(json.dumps(r) + '\n')
s = r['engine_stats_rank0']
print(sys.argv[1], r['value'], 'p50', r.get('p50_latency_ms'), 'dev', r['device_ms_p50'],
      'cores', r['cpu_cores_busy_rank0'], {k: s.get(k) for k in (
          'pinned_chunks', 'pinned_in_use_max', 'pinned_waits', 'pinned_wait_s',
          'pinned_heap_budget', 'queue_records', 'ingested_records', 'records_in',
          'thread_s_ingest', 'thread_s_decode', 'thread_s_wait', 'batch_images_mean')}, flush=True)
PY
done
export TMPDIR=/tmp
# one hardware queue per HIP stream under the profiler: its queue interception crashed when the
# engine's streams (replicas + ingest lanes, > 4 from several threads) shared HIP's default 4
# (a SIGSEGV inside librocprofiler-sdk under GpuIngest::run, gpurun_out/final/prof_bench.log);
# the same setting gale's --profile uses
export GPU_MAX_HW_QUEUES=32
timeout -k 10 300 rocprofv3 --kernel-trace -d $d/prof -o run -- \
    python bench.py --model resnet50 --steps 10 --warmup 3 --latency-load 0 > $d/prof.log 2>&1 || exit 1
python tools/prof_summary.py $(find $d/prof -name '*.db' | head -1) --busy --top 14 > $d/busy.txt
cat $d/busy.txt
rm -rf $d/prof
