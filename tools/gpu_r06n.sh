#!/bin/bash
# round 6, call n: launch shapes of the f32 conv / wgrad / finalize kernels and the 16-bit halo / up-2 kernels
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 rocprofv3 --kernel-trace -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-roofline --steps 16 > "$O/prof_bench.log" 2>&1 || { echo PFAIL; tail -20 $O/prof_bench.log; exit 1; }
t=$(find "$O/prof" -name 'run_kernel_trace.csv' | head -1)
python3 tools/trace_kstats.py "$t" 'conv_fwd_kernel<float|conv_wgrad_kernel<float|finalize' 40 > $O/f32_shapes.txt
python3 tools/trace_kstats.py "$t" 'halo_kernel|up2_kernel|s2g|c64p|c64r' 40 > $O/c16_shapes.txt
python3 tools/trace_kstats.py "$t" 'wgrad3x3' 30 > $O/w16_shapes.txt
rm -f "$t"
cat $O/f32_shapes.txt
