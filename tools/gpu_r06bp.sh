#!/bin/bash
# round 6, call bp: the 4x4 FIR strip kernel's C = 32 form -- FIR tests, C5 A/B (SG2_FIR_C32), C2 bench
set -o pipefail
O=gpurun_out/r06bp
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "upfirdn or fir" > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
TAG=r06bp CFG=c5 VAR=SG2_FIR_C32 VALS="- 0" bash tools/gpu_sweep_cfg.sh || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $O/bench_c2.log 2>&1 || { echo BFAIL; tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c1-120
