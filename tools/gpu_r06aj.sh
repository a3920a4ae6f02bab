#!/bin/bash
# round 6, call aj: 1-D FIR pass grid size A/B (workgroups looping over more (row, tile) pairs)
set -o pipefail
O=gpurun_out/r06aj
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for g in 16384 4096 2048 1024; do
SG2_U1D_GRID=$g timeout -k 10 200 python -u tools/ada_micro.py 40 det > $O/ada_det_$g.txt 2>&1 || { echo AFAIL; tail -20 $O/ada_det_$g.txt; exit 1; }
echo "grid=$g"; grep -E "ADA|upfirdn" $O/ada_det_$g.txt
done
