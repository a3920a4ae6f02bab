#!/bin/bash
# round 6, call bc: the final tree (with the parameter-layout wgrad test) -- full GPU suite in the driver's order, smoke
set -o pipefail
O=gpurun_out/r06bc
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 780 python -u -m pytest tests/ -x -v -m gpu --timeout 450 --timeout-method thread --durations=15 > $O/pytest_gpu.log 2>&1 || { echo TFAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SFAIL; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
