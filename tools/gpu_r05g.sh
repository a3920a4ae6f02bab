#!/bin/bash
# round 5, call g: multi-pack v3 tests, bench + profile with ring 49 default
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_trainer_gpu.py -k "pack" > $O/t1.log 2>&1 || { echo T1FAIL; tail -40 $O/t1.log; exit 1; }
tail -1 $O/t1.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "pack_weight or c64_ring and 49 and mod_epi_raw" > $O/t2.log 2>&1 || { echo T2FAIL; tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --steps 16 > "$O/prof_bench.log" 2>&1 || { echo PFAIL; tail -20 $O/prof_bench.log; exit 1; }
f=$(find "$O/prof" -name 'run_kernel_stats.csv' | head -1)
python3 "$R/profiles/prof_summary.py" "$(dirname "$f")" 45 > "$O/prof_summary.txt" 2>&1
ms=$(python3 -c "import json,sys; print(json.loads([l for l in open('$O/prof_bench.log') if l.startswith('{')][-1])['ms_per_step'])")
t=$(find "$O/prof" -name 'run_kernel_trace.csv' | head -1)
python3 "$R/profiles/step_breakdown.py" "$t" "$ms" > "$O/step_breakdown.txt" 2>&1; head -24 "$O/step_breakdown.txt"
rm -f "$t"
grep -i "pack\|c64r" $O/prof_summary.txt | head -6
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { echo BFAIL; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
