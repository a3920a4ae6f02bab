#!/bin/bash
# round 6, call ae: ADA micro in the deterministic default
set -o pipefail
O=gpurun_out/r06ae
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 python -u tools/ada_micro.py 40 det > $O/ada_det.txt 2>&1 || { echo AFAIL; tail -20 $O/ada_det.txt; exit 1; }
grep -E "ADA|us/iter" $O/ada_det.txt | head -14
