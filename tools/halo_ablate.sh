#!/bin/bash
# Ablation of the halo conv kernel (SG2_HALO_DBG bits, conv3x3.hip): which part bounds it.
for d in 0 1 2 4 8 3 6 12 14; do
  echo "dbg=$d: $(SG2_HALO_DBG=$d timeout -k 5 60 python3 tools/conv_micro.py --which halo --reps 10 2>/dev/null | grep -v amdgpu | tr '\n' ' ' | sed 's/halo-fused+raw [0-9.]*ms | //g')"
done
