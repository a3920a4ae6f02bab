#!/bin/bash
# round 6, call f: the configuration tests in the production (deterministic) arithmetic, with durations
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -q -rA --durations=40 --timeout 400 --timeout-method thread -m gpu \
    tests/test_config_gpu.py > $O/config_tests.log 2>&1
rc=$?
cp gpurun_out/config_parity.jsonl $O/ 2>/dev/null
grep -E "PASSED|FAILED|passed|failed|^[0-9.]+s call" $O/config_tests.log | tail -60
exit $rc
