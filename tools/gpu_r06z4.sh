#!/bin/bash
# round 6, call z4: ADA FIR / zero-region changes in the step -- bench-step tests, bench x2
set -o pipefail
O=gpurun_out/r06z4
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_bench_gpu.py > $O/tb.log 2>&1 || { echo BTFAIL; tail -30 $O/tb.log; exit 1; }
tail -1 $O/tb.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$i.log 2>&1 || { echo BFAIL; tail -20 $O/bench_$i.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
