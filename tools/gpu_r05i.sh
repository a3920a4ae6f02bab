#!/bin/bash
# round 5, call i: the C = 32 ring kernel (parity, then the C5 bench whose roofline layer is 1024^2 C=32)
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "c32_ring" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 400 python -u bench.py --res 1024 --batch-gpu 8 --img-channels 3 --cbase 32768 --c-dim 0 --fp16-dtype bf16 --steps 32 --warmup 8 --no-cpu-baseline > $O/c5_ring.log 2>&1 || { tail -20 $O/c5_ring.log; exit 1; }
tail -1 $O/c5_ring.log | cut -c1-1500
SG2_C32_RING=0 timeout -k 10 400 python -u bench.py --res 1024 --batch-gpu 8 --img-channels 3 --cbase 32768 --c-dim 0 --fp16-dtype bf16 --steps 32 --warmup 8 --no-cpu-baseline > $O/c5_noring.log 2>&1 || { tail -20 $O/c5_noring.log; exit 1; }
tail -1 $O/c5_noring.log | cut -c1-600
