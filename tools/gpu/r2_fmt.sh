set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/fmt_bench.py 2560 && timeout -k 10 120 python tools/fmt_bench.py 40960
