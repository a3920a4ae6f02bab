#!/bin/bash
# round 6, call ay: up-2 conv workgroup order A/B (micro + bench), up-2 tests
set -o pipefail
O=gpurun_out/r06ay
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 python -u tools/up2_order_ab.py > $O/up2_order_ab.txt 2>&1 || { echo UFAIL; tail -20 $O/up2_order_ab.txt; exit 1; }
cat $O/up2_order_ab.txt | grep N=
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ -k "up2 or up_2 or upconv or Up" > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
for o in 1 0; do
SG2_UP2_ORDER=$o timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $O/bench_o${o}_$i.log 2>&1 || { echo BFAIL; tail -20 $O/bench_o${o}_$i.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_o${o}_$i.log') if l.startswith('{')][-1]); print('order $o', d['value'], d['ms_per_step'])"
done
done
