#!/bin/bash
# round 5, call h: configuration-width parity (f32 det / atomic / exact, 16-bit det / atomic)
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
export PYTHONUNBUFFERED=1
rm -f gpurun_out/config_parity.jsonl
timeout -k 10 1100 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_config_gpu.py > $O/t.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $O/t.log | sed 's/.*test_config_gpu.py:://' | cut -c1-150
tail -3 $O/t.log
cp gpurun_out/config_parity.jsonl $O/ 2>/dev/null
exit $rc
