#!/bin/bash
for nb in 1 2; do
  echo "nbuf=$nb: $(SG2_HALO_NBUF=$nb timeout -k 5 60 python3 tools/conv_micro.py --which halo --reps 10 2>/dev/null | grep -v amdgpu | tr '\n' ' ' | sed 's/halo-fused+raw [0-9.]*ms | //g')"
done
