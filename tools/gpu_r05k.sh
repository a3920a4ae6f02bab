#!/bin/bash
# round 5, call k: the product's own 16-bit spread under f32-ulp state nudges (C2 bf16 / fp16) and the pack census
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/nudge16.py c2 bf16 6 > $O/nudge_c2_bf16.log 2>&1 || { tail -30 $O/nudge_c2_bf16.log; exit 1; }
tail -16 $O/nudge_c2_bf16.log
timeout -k 10 200 python -u tools/nudge16.py c2 fp16 3 > $O/nudge_c2_fp16.log 2>&1 || { tail -30 $O/nudge_c2_fp16.log; exit 1; }
tail -4 $O/nudge_c2_fp16.log
timeout -k 10 300 python -u tools/pack_census.py > $O/pack_census.log 2>&1 || { tail -30 $O/pack_census.log; exit 1; }
head -30 $O/pack_census.log
