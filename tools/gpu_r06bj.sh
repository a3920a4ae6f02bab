#!/bin/bash
# round 6, call bj: where the library's zero fills go (kernel trace of a short bench)
set -o pipefail
O=gpurun_out/r06bj
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-roofline --steps 16 --warmup 8 > "$O/prof_bench.log" 2>&1 || { echo PFAIL; tail -20 $O/prof_bench.log; exit 1; }
t=$(find "$O/prof" -name 'run_kernel_trace.csv' | head -1)
python3 tools/zero_fill_sites.py "$t" 26 > $O/zero_fill_sites.txt 2>&1; cat $O/zero_fill_sites.txt
rm -f "$t"
