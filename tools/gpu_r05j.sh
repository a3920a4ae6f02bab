#!/bin/bash
# round 5, call j: Dreg 16-bit scale diagnostic (C2) and the conv census of the default bench step
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/dreg_diag.py c2 > $O/dreg_diag.log 2>&1 || { tail -30 $O/dreg_diag.log; exit 1; }
grep -v "^ *[0-9]* b\|hook" $O/dreg_diag.log | tail -30
timeout -k 10 400 python -u tools/conv_census.py > $O/conv_census.log 2>&1 || { tail -30 $O/conv_census.log; exit 1; }
head -40 $O/conv_census.log
