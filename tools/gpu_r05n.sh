#!/bin/bash
# round 5, call n: configuration parity (16-bit distributions, f32), bench + rocprof step breakdown
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
export PYTHONUNBUFFERED=1
rm -f gpurun_out/config_parity.jsonl
timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_config_gpu.py > $O/t.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $O/t.log | sed 's/.*test_config_gpu.py:://' | cut -c1-200
cp gpurun_out/config_parity.jsonl $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --steps 16 > "$O/prof_bench.log" 2>&1 || { echo PFAIL; tail -20 $O/prof_bench.log; exit 1; }
f=$(find "$O/prof" -name 'run_kernel_stats.csv' | head -1)
python3 "$R/profiles/prof_summary.py" "$(dirname "$f")" 45 > "$O/prof_summary.txt" 2>&1
ms=$(python3 -c "import json,sys; print(json.loads([l for l in open('$O/prof_bench.log') if l.startswith('{')][-1])['ms_per_step'])")
t=$(find "$O/prof" -name 'run_kernel_trace.csv' | head -1)
python3 "$R/profiles/step_breakdown.py" "$t" "$ms" > "$O/step_breakdown.txt" 2>&1; head -30 "$O/step_breakdown.txt"
rm -f "$t"
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { echo BFAIL; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 300 python -u tools/nudge16.py c2 bf16 6 > $O/nudge_c2_bf16.log 2>&1 || { tail -30 $O/nudge_c2_bf16.log; exit 1; }
grep -v amdgpu.ids $O/nudge_c2_bf16.log | tail -20
