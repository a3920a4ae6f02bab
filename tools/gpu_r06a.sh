#!/bin/bash
# round 6, call a: C4 f32 det-vs-atomic attribution; bench cost of deterministic mode (alternating A/B)
set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 420 python -u tools/atomic_attr.py c4 4 > $O/attr_c4.log 2>&1 || { echo AFAIL; tail -30 $O/attr_c4.log; exit 1; }
for m in off on off on; do
  timeout -k 10 300 python -u bench.py --steps 48 --no-cpu-baseline --no-roofline --deterministic $m > $O/bench_det_$m.log 2>&1 || { echo BFAIL $m; tail -20 $O/bench_det_$m.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_det_$m.log') if l.startswith('{')][-1]); print('det', '$m', d['value'], d['ms_per_step'])"
done
