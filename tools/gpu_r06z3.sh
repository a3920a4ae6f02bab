#!/bin/bash
# round 6, call z3: ADA FIR horizontal passes staged in LDS (A/B), zero region skipped under the det gather
set -o pipefail
O=gpurun_out/r06z3
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_deterministic_gpu.py \
    -k "upfirdn or augment or fir or grid_sample or dynamic or det" > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0; do
  SG2_U1D_HLDS=$v timeout -k 10 200 python -u tools/ada_micro.py > $O/ada_$v.txt 2>&1 || { echo AFAIL; tail -20 $O/ada_$v.txt; exit 1; }
  echo "hlds=$v"; grep -E "ADA|upfirdn|zero" $O/ada_$v.txt
done
