#!/bin/bash
# round 6, call g: the whole GPU suite in the driver's order (-x, no exclusions), with durations; then smoke
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1080 python -u -m pytest tests/ -x -q -m gpu --durations=60 --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -75 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; tail -2 $O/smoke.log
