# list the PMC counters rocprofv3 offers on this GPU (names for the --pmc passes)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --list-avail > gpurun_out/counters.txt 2>&1 || timeout -s KILL 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
grep -oE "(SQ|TCC|TCP|TA|TD|GRBM)_[A-Z0-9_]+" gpurun_out/counters.txt | sort -u > gpurun_out/counter_names.txt
wc -l gpurun_out/counter_names.txt
grep -E "MFMA|LDS_BANK|SQ_WAVES$|BUSY_CYCLES|FETCH|WRITE|TCC_HIT|TCC_MISS|OCCUP" gpurun_out/counter_names.txt | head -60
