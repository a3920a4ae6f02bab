#!/bin/bash
# round 5, call ah: the training-loop end-to-end test (metric registry rewrite) and smoke on the final tree
set -o pipefail
O=gpurun_out/r05ah
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -v --timeout 650 --timeout-method thread tests/test_training_loop_gpu.py > $O/loop.log 2>&1 || { tail -40 $O/loop.log; exit 1; }
tail -3 $O/loop.log
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
