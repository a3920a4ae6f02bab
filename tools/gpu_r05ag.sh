#!/bin/bash
# round 5, call af: C4 same-state 16-bit parity (seeds 1-4)
set -o pipefail
O=gpurun_out/r05ag
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_config_gpu.py -k "16bit and c4" > $O/c4_16.log 2>&1 || { tail -40 $O/c4_16.log; exit 1; }
tail -2 $O/c4_16.log
