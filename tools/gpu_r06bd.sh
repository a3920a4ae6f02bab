#!/bin/bash
# round 6, call bd: the 8-wave 16 x 16-cell up-2 conv form -- parity tests, micro A/B, bench A/B
set -o pipefail
O=gpurun_out/r06bd
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "up2" > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/up2_wide_ab.py > $O/up2_wide_ab.txt 2>&1 || { echo UFAIL; tail -20 $O/up2_wide_ab.txt; exit 1; }
grep N= $O/up2_wide_ab.txt
for i in 1 2; do
for wv in 1 0; do
SG2_UP2_WIDE=$wv timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $O/bench_w${wv}_$i.log 2>&1 || { echo BFAIL; tail -20 $O/bench_w${wv}_$i.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_w${wv}_$i.log') if l.startswith('{')][-1]); print('wide $wv', d['value'], d['ms_per_step'])"
done
done
