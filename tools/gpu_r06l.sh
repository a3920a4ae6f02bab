#!/bin/bash
# round 6, call l: layer_bwd deterministic combine in-launch vs det_sum launches, same box, alternating
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for c in 1 0 1 0 1 0; do
  SG2_LB_COMBINE=$c timeout -k 10 300 python -u bench.py --steps 64 --no-cpu-baseline --no-roofline > $O/bench_$c.log 2>&1 || { echo BFAIL; tail -20 $O/bench_$c.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_$c.log') if l.startswith('{')][-1]); print('combine', '$c', d['value'], d['ms_per_step'])" | tee -a $O/ab.txt
done
