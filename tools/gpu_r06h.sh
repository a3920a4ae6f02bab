#!/bin/bash
# round 6, call h: ring form 50 (DMAs spread over the tap loop) -- parity, A/B against 49
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py \
    -k "test_conv3x3_c64_ring and (49 or 50)" > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 49 50 49 50 49 50; do
  SG2_C64_RING=$r timeout -k 10 120 python -u tools/ring_ab.py 5 2>&1 | grep -v amdgpu.ids | head -1 | tee -a $O/ab.log
done
