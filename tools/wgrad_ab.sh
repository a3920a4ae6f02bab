#!/bin/bash
for sw in 0 1 0 1; do
  echo "swz=$sw: $(SG2_WGRAD_SWZ=$sw timeout -k 5 60 python3 tools/conv_micro.py --which wgrad,halo --reps 10 2>/dev/null | grep -v amdgpu | tr '\n' ' ' | sed 's/halo-fused+raw [0-9.]*ms | //g')"
done
