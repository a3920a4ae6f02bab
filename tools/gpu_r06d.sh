#!/bin/bash
# round 6, call d: where the deterministic mode's reductions go (det_sum per launch shape, wgrad kernels)
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 rocprofv3 --kernel-trace -d "$O/prof_on" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-roofline --steps 16 --deterministic on > "$O/prof_bench_on.log" 2>&1 || { echo PFAIL; tail -20 $O/prof_bench_on.log; exit 1; }
t=$(find "$O/prof_on" -name 'run_kernel_trace.csv' | head -1)
head -1 "$t" > $O/trace_header.txt
python3 tools/trace_kstats.py "$t" 'det_sum|finalize|gather' 40 > $O/det_shapes.txt
python3 tools/trace_kstats.py "$t" 'wgrad' 40 > $O/wgrad_shapes.txt
rm -f "$t"
cat $O/trace_header.txt $O/det_shapes.txt $O/wgrad_shapes.txt
