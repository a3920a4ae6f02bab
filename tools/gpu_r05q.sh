#!/bin/bash
# round 5, call q: the halo kernel's direct epilogue (parity, A/B) and the bench
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "halo_direct or conv3x3_fused or conv3x3_dot or fused_d_conv or fused_synthesis or layer_vjp or conv3x3_s2 or c32_ring" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python -u tools/halo_direct_ab.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { echo BFAIL; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
