#!/bin/bash
# round 6, call at: staged sums (no memsets in the step) -- memset inventory, full GPU suite in driver order, smoke, bench
set -o pipefail
O=gpurun_out/r06at
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 python -u tools/memset_ops.py > $O/memset_ops.txt 2>&1 || { echo MFAIL; tail -20 $O/memset_ops.txt; exit 1; }
head -3 $O/memset_ops.txt
timeout -k 10 780 python -u -m pytest tests/ -x -v -m gpu --timeout 450 --timeout-method thread --durations=15 > $O/pytest_gpu.log 2>&1 || { echo TFAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SFAIL; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 240 python -u bench.py > $O/bench.log 2>&1 || { echo BFAIL; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
