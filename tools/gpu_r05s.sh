#!/bin/bash
# round 5, call s: the GPU suite (all but the 16-bit config tests, whose fixtures are being extended), smoke, C4 bench
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "not test_16bit_phases" > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 500 python -u bench.py --res 512 --batch-gpu 16 --img-channels 3 --cbase 32768 --c-dim 0 > $O/c4_bench.log 2>&1 || { tail -20 $O/c4_bench.log; exit 1; }
tail -1 $O/c4_bench.log | cut -c1-300
