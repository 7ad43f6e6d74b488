# does the end-to-end rate decay over a long window? (per-step rates of a 60-step run)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 60 --warmup 5 > gpurun_out/long.json 2> gpurun_out/long.err || { tail -20 gpurun_out/long.err; exit 1; }
python -c "import json;r=json.load(open('gpurun_out/long.json'));print(r['value'],r['timed_s'],r['cpu_cores_by_stage_rank0']);print(r['step_rates'])"
