#!/bin/bash
# round 6, call j: layer_bwd forms A/B (pixels in flight, non-temporal stores), f16 and det
set -o pipefail
O=gpurun_out/r06j
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for f in 0 1 2 0 1 2; do
  SG2_LB_FORM=$f timeout -k 10 120 python -u tools/lb_micro.py 2>&1 | grep -v amdgpu.ids | tee -a $O/lb_ab.log | grep "C=64 "
done
