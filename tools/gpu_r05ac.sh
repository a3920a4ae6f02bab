#!/bin/bash
# round 5, call ac: GPU suite (all but the 16-bit config tests), smoke after the up-2 edge split
set -o pipefail
O=gpurun_out/r05ac
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "not test_16bit_phases" > $O/pytest_gpu.log 2>&1
rc=$?
tail -4 $O/pytest_gpu.log
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
exit $rc
exit $rc
