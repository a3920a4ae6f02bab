#!/bin/bash
# round 6, call ah: horizontal 1-D FIR segments 256 vs 128 wide (2 rows a workgroup) -- parity, det ADA micro
set -o pipefail
O=gpurun_out/r06ah
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for w in 128 256; do
SG2_U1D_HTW=$w timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_deterministic_gpu.py \
    -k "upfirdn or augment or dynamic or gather" > $O/tests_$w.log 2>&1 || { echo TFAIL; tail -30 $O/tests_$w.log; exit 1; }
tail -1 $O/tests_$w.log
SG2_U1D_HTW=$w timeout -k 10 200 python -u tools/ada_micro.py 40 det > $O/ada_det_$w.txt 2>&1 || { echo AFAIL; tail -20 $O/ada_det_$w.txt; exit 1; }
echo "htw=$w"; grep -E "ADA|upfirdn" $O/ada_det_$w.txt
done
