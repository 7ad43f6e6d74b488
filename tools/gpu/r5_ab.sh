#!/bin/bash
# Round-5 interleaved A/B on ONE box: ARMS="name:args|name:args|..." run REPS times each, in
# turn; every JSON line to gpurun_out/ab/runs${TAG}.jsonl with its label; a one-line summary per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/ab
mkdir -p $out
runs=$out/runs${TAG:+_$TAG}.jsonl
: > $runs
IFS='|' read -ra arms <<< "$ARMS"
for i in $(seq 1 ${REPS:-3}); do
  for arm in "${arms[@]}"; do
    name=${arm%%:*}
    args=${arm#*:}
    timeout -k 10 ${SECS:-240} python bench.py $args > $out/one.jsonl 2> $out/${name}_$i.err || {
      echo "FAILED $name"; tail -5 $out/${name}_$i.err; exit 1; }
    python - "${name}_$i" "$runs" <<'PY'
import json, sys
r = json.loads(open('gpurun_out/ab/one.jsonl').read().strip().splitlines()[-1])
r['label'] = sys.argv[1]
open(sys.argv[2], 'a').write(json.dumps(r) + '\n')
print(sys.argv[1], r['value'], 'p50', r.get('p50_latency_ms'), 'p99', r.get('p99_latency_ms'),
      'p999', r.get('p999_latency_ms'), 'dev', r['device_ms_p50'],
      'cores', r['cpu_cores_busy_rank0'], r['cpu_cores_by_stage_rank0'],
      'spread', r['step_rate_spread']['range_pct'], 'thr', r['timed_cgroup_rank0'].get('throttled_ms'),
      flush=True)
PY
  done
done
