#!/bin/bash
# round 5, call t: GPU suite (all but the 16-bit config tests), smoke, glue census
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "not test_16bit_phases" > $O/pytest_gpu.log 2>&1
rc=$?
tail -4 $O/pytest_gpu.log
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python -u tools/glue_census.py > $O/glue_census.log 2>&1 || { tail -20 $O/glue_census.log; exit 1; }
head -60 $O/glue_census.log
exit $rc
