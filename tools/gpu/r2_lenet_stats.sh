# where does LeNet-5 under backlog spend its ~1 s fetch -> ack? (all engine stats)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model lenet5 --all-stats > gpurun_out/ls.json 2> gpurun_out/ls.err || { tail -8 gpurun_out/ls.err; exit 1; }
python -c "import json;r=json.load(open('gpurun_out/ls.json'));print(r['value'], r['p50_latency_ms']);print(json.dumps(r['engine_stats_rank0']))"
timeout -k 10 300 python bench.py --all-stats > gpurun_out/rs.json 2> gpurun_out/rs.err || { tail -8 gpurun_out/rs.err; exit 1; }
python -c "import json;r=json.load(open('gpurun_out/rs.json'));print(r['value'], r['p50_latency_ms']);print(json.dumps(r['engine_stats_rank0']))"
