#!/bin/bash
# round 5, call aa: the ring's dynamic-tail share (SG2_RING_DYN) after the division-free decode
set -o pipefail
O=gpurun_out/r05aa
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for d in 12 16 20 24 8; do
    SG2_RING_DYN=$d timeout -k 10 120 python -u tools/ring_ab.py 5 > $O/dyn${d}_$rep.log 2>&1 || { tail -5 $O/dyn${d}_$rep.log; exit 1; }
    echo "dyn=$d $(grep 'fused launch' $O/dyn${d}_$rep.log)"
  done
done
