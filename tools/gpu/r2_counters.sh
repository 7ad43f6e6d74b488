# PMC counter names offered on this GPU (written to gpurun_out/counter_names.txt)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
grep -oE "(SQ|TCC|TCP|TA|TD|GRBM|SPI)_[A-Z0-9_]+" gpurun_out/counters.txt | sort -u > gpurun_out/counter_names.txt
wc -l gpurun_out/counter_names.txt
