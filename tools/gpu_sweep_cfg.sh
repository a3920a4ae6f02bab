#!/bin/bash
# Bench A/B over values of one environment switch on a named configuration (c4 / c5), alternating, two rounds:
#   gpurun -- 'TAG=<tag> CFG=c5 VAR=<name> VALS="<v1> <v2>" bash tools/gpu_sweep_cfg.sh'   ("-": switch unset)
set -o pipefail
O=gpurun_out/${TAG:?}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ "${CFG:?}" = c4 ]; then A="--res 512 --batch-gpu 16 --img-channels 3 --cbase 32768 --c-dim 0"
else A="--res 1024 --batch-gpu 8 --img-channels 3 --cbase 32768 --c-dim 0 --fp16-dtype bf16"; fi
for i in 1 2; do
for v in ${VALS:?}; do
if [ "$v" = "-" ]; then envs=""; else envs="$VAR=$v"; fi
env $envs timeout -k 10 400 python -u bench.py $A --no-cpu-baseline --no-roofline > $O/bench_${CFG}_${VAR}_${v}_$i.log 2>&1 || { echo BFAIL; tail -20 $O/bench_${CFG}_${VAR}_${v}_$i.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_${CFG}_${VAR}_${v}_$i.log') if l.startswith('{')][-1]); print('$CFG $VAR=$v', d['value'], d['ms_per_step'])"
done
done
