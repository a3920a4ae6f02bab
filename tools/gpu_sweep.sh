#!/bin/bash
# Bench A/B over values of one environment switch, alternating, two rounds:
#   gpurun -- 'TAG=<tag> VAR=<name> VALS="<v1> <v2> ..." bash tools/gpu_sweep.sh'   (VAR unset for a value: "-")
set -o pipefail
O=gpurun_out/${TAG:?}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2; do
for v in ${VALS:?}; do
if [ "$v" = "-" ]; then envs=""; else envs="$VAR=$v"; fi
env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $O/bench_${VAR}_${v}_$i.log 2>&1 || { echo BFAIL; tail -20 $O/bench_${VAR}_${v}_$i.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_${VAR}_${v}_$i.log') if l.startswith('{')][-1]); print('$VAR=$v', d['value'], d['ms_per_step'])"
done
done
