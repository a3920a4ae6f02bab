#!/bin/bash
# round 6, call bk: deterministic slot sums assign their accumulators (no zero fills) -- det / op tests first, then
# the full GPU suite in the driver's order, smoke, bench A/B (SG2_DET_ASSIGN), fill census
set -o pipefail
O=gpurun_out/r06bk
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$(pwd)
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_deterministic_gpu.py tests/test_bench_gpu.py > $O/tests_det.log 2>&1 || { echo DFAIL; tail -30 $O/tests_det.log; exit 1; }
tail -1 $O/tests_det.log
timeout -k 10 780 python -u -m pytest tests/ -x -v -m gpu --timeout 450 --timeout-method thread --durations=15 > $O/pytest_gpu.log 2>&1 || { echo TFAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SFAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
TAG=r06bk VAR=SG2_DET_ASSIGN VALS="- 0" bash tools/gpu_sweep.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-roofline --steps 16 --warmup 8 > "$O/prof_bench.log" 2>&1 || { echo PFAIL; tail -20 $O/prof_bench.log; exit 1; }
t=$(find "$O/prof" -name 'run_kernel_trace.csv' | head -1)
python3 tools/zero_fill_sites.py "$t" 26 > $O/zero_fill_sites.txt 2>&1; head -3 $O/zero_fill_sites.txt
rm -f "$t"
