#!/bin/bash
# round 6, call ak: grid-size A/B of the deterministic gather and the reflect pad
set -o pipefail
O=gpurun_out/r06ak
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for g in 16384 8192 4096 2048; do
SG2_GATHER_GRID=$g SG2_PAD_GRID=$g timeout -k 10 200 python -u tools/ada_micro.py 40 det > $O/ada_det_$g.txt 2>&1 || { echo AFAIL; tail -20 $O/ada_det_$g.txt; exit 1; }
echo "grid=$g"; grep -E "ADA|gather|reflect" $O/ada_det_$g.txt
done
