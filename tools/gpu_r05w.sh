#!/bin/bash
# round 5, call w: the 16-bit configuration tests (same-state C2 bf16 samples merged)
set -o pipefail
O=gpurun_out/r05w
mkdir -p $O
export PYTHONUNBUFFERED=1
rm -f gpurun_out/config_parity.jsonl
timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_config_gpu.py -k "test_16bit_phases" > $O/t.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $O/t.log | sed 's/.*test_config_gpu.py:://' | cut -c1-200
grep -E "^E  " $O/t.log | cut -c1-400 | head -6
cp gpurun_out/config_parity.jsonl $O/ 2>/dev/null
exit $rc
