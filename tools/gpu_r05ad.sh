#!/bin/bash
# round 5, call ad: every 16-bit config test (same-state fixtures for C1 and C2) after the up-2 edge split
set -o pipefail
O=gpurun_out/r05ad
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python -u -m pytest tests/test_config_gpu.py -v --timeout 400 --timeout-method thread -k "test_16bit_phases" > $O/config16.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/config16.log | tail -25
exit $rc
