#!/bin/bash
# round 6, call z2: 1-D FIR passes, grid-strided with compile-time up/down (vertical runs on / off) -- parity, ADA micro
set -o pipefail
O=gpurun_out/r06z2
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py \
    -k "upfirdn or augment or fir or grid_sample or dynamic" > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 4 0; do
  SG2_U1D_VRUN=$v timeout -k 10 200 python -u tools/ada_micro.py > $O/ada_$v.txt 2>&1 || { echo AFAIL; tail -20 $O/ada_$v.txt; exit 1; }
  echo "vrun=$v"; grep -E "ADA|upfirdn" $O/ada_$v.txt
done
