#!/bin/bash
# round 5, call f: multi-pack v2 + ring 49 (per-sample dynamic tail): parity, A/B, stamps, bench + profile
set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_trainer_gpu.py -k "pack" > $O/t1.log 2>&1 || { echo T1FAIL; tail -40 $O/t1.log; exit 1; }
tail -1 $O/t1.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "c64_ring and (49 or 46)" > $O/t2.log 2>&1 || { echo T2FAIL; tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
for rep in 1 2; do for f in 46 49; do
  SG2_C64_RING=$f timeout -k 10 120 python -u tools/ring_ab.py 3 2>&1 | grep -v amdgpu | head -1 >> $O/ring_ab.log || { echo RABFAIL; exit 1; }
done; for d in 6 20; do
  SG2_RING_DYN=$d SG2_C64_RING=49 timeout -k 10 120 python -u tools/ring_ab.py 3 2>&1 | grep -v amdgpu | head -1 | sed "s/^/dyn$d /" >> $O/ring_ab.log || { echo RABFAIL; exit 1; }
done; done
cat $O/ring_ab.log
SG2_C64_RING=49 SG2HIP_LIB=tools/diag_libs/libsg2hip_r512.so timeout -k 10 120 python -u tools/ring_stamps.py > $O/stamps_49.log 2>&1 || { echo STFAIL; tail -20 $O/stamps_49.log; exit 1; }
grep -v amdgpu $O/stamps_49.log
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --steps 16 > "$O/prof_bench.log" 2>&1 || { echo PFAIL; tail -20 $O/prof_bench.log; exit 1; }
f=$(find "$O/prof" -name 'run_kernel_stats.csv' | head -1)
python3 "$R/profiles/prof_summary.py" "$(dirname "$f")" 45 > "$O/prof_summary.txt" 2>&1
ms=$(python3 -c "import json,sys; print(json.loads([l for l in open('$O/prof_bench.log') if l.startswith('{')][-1])['ms_per_step'])")
t=$(find "$O/prof" -name 'run_kernel_trace.csv' | head -1)
python3 "$R/profiles/step_breakdown.py" "$t" "$ms" > "$O/step_breakdown.txt" 2>&1; head -16 "$O/step_breakdown.txt"
rm -f "$t"
grep -i pack $O/prof_summary.txt | head -4
