#!/bin/bash
# round 6, call ad: ADA micro in the deterministic default; vertical FIR runs of 4 vs 8 rows
set -o pipefail
O=gpurun_out/r06ad
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in 4 8; do
  SG2_U1D_VRUN=$v timeout -k 10 200 python -u tools/ada_micro.py 40 det > $O/ada_det_$v.txt 2>&1 || { echo AFAIL; tail -20 $O/ada_det_$v.txt; exit 1; }
  echo "vrun=$v"; grep -E "ADA|upfirdn|grid|zero|pad" $O/ada_det_$v.txt
done
SG2_U1D_VRUN=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py \
    -k "upfirdn or augment or dynamic" > $O/tests8.log 2>&1 || { echo TFAIL; tail -30 $O/tests8.log; exit 1; }
tail -1 $O/tests8.log
