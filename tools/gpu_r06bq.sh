#!/bin/bash
# round 6, call bq: final tree with the C = 32 FIR form -- full GPU suite in the driver's order, smoke, bench,
# order, smoke, bench, rocprof step breakdown, C4 / C5 lines
set -o pipefail
O=gpurun_out/r06bq
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$(pwd)
timeout -k 10 780 python -u -m pytest tests/ -x -v -m gpu --timeout 450 --timeout-method thread --durations=15 > $O/pytest_gpu.log 2>&1 || { echo TFAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SFAIL; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo BFAIL; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --steps 16 > "$O/prof_bench.log" 2>&1 || { echo PFAIL; tail -20 $O/prof_bench.log; exit 1; }
f=$(find "$O/prof" -name 'run_kernel_stats.csv' | head -1)
python3 "$R/profiles/prof_summary.py" "$(dirname "$f")" 45 > "$O/prof_summary.txt" 2>&1
ms=$(python3 -c "import json,sys; print(json.loads([l for l in open('$O/prof_bench.log') if l.startswith('{')][-1])['ms_per_step'])")
t=$(find "$O/prof" -name 'run_kernel_trace.csv' | head -1)
python3 "$R/profiles/step_breakdown.py" "$t" "$ms" > "$O/step_breakdown.txt" 2>&1; head -12 "$O/step_breakdown.txt"
rm -f "$t"
timeout -k 10 500 python -u bench.py --res 512 --batch-gpu 16 --img-channels 3 --cbase 32768 --c-dim 0 --no-cpu-baseline > $O/c4_bench.log 2>&1 || { tail -20 $O/c4_bench.log; exit 1; }
tail -1 $O/c4_bench.log | cut -c1-200
timeout -k 10 500 python -u bench.py --res 1024 --batch-gpu 8 --img-channels 3 --cbase 32768 --c-dim 0 --fp16-dtype bf16 --no-cpu-baseline > $O/c5_bench.log 2>&1 || { tail -20 $O/c5_bench.log; exit 1; }
tail -1 $O/c5_bench.log | cut -c1-200
