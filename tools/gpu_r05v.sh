#!/bin/bash
# round 5, call v: kernel-path A/B of the C2 bf16 Dreg result at three states
set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u tools/dreg_ab.py 0 1 2 3 4 > $O/dreg_ab.log 2>&1 || { tail -20 $O/dreg_ab.log; exit 1; }
tail -3 $O/dreg_ab.log
