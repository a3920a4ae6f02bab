#!/bin/bash
# round 6, call be: the f32 weight-gradient split target (SG2_CWGRAD_WGS) after the parameter-layout slot sum
set -o pipefail
O=gpurun_out/${TAG:-r06be}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2; do
for v in ${VALS:-2048 1024 4096}; do
SG2_CWGRAD_WGS=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $O/bench_c${v}_$i.log 2>&1 || { echo BFAIL; tail -20 $O/bench_c${v}_$i.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_c${v}_$i.log') if l.startswith('{')][-1]); print('cwgrad $v', d['value'], d['ms_per_step'])"
done
done
