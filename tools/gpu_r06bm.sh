#!/bin/bash
# round 6, call bm: step breakdowns of the C4 (512^2 3-ch bs16) and C5 (1024^2 3-ch bs8 bf16) configurations
set -o pipefail
O=gpurun_out/r06bm
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$(pwd)
for c in c4 c5; do
if [ $c = c4 ]; then A="--res 512 --batch-gpu 16 --img-channels 3 --cbase 32768 --c-dim 0"; else A="--res 1024 --batch-gpu 8 --img-channels 3 --cbase 32768 --c-dim 0 --fp16-dtype bf16"; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_$c" -o run --output-format csv \
    -- python3 "$R/bench.py" $A --no-cpu-baseline --no-roofline --steps 16 > "$O/prof_${c}_bench.log" 2>&1 || { echo PFAIL; tail -20 $O/prof_${c}_bench.log; exit 1; }
ms=$(python3 -c "import json,sys; print(json.loads([l for l in open('$O/prof_${c}_bench.log') if l.startswith('{')][-1])['ms_per_step'])")
t=$(find "$O/prof_$c" -name 'run_kernel_trace.csv' | head -1)
python3 "$R/profiles/step_breakdown.py" "$t" "$ms" > "$O/${c}_step_breakdown.txt" 2>&1; head -12 "$O/${c}_step_breakdown.txt"
rm -f "$t"
done
