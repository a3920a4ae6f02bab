#!/bin/bash
# round 5, call a: new tests, ring forms (parity + A/B), ring stamps (diag lib), bench default
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py \
  -k "sign_nan or vjp_nodes_upstream or training_stats_moments or demod_kernel or infnorm_prenorm or (c64_ring and (45 or 46 or 47))" > $O/t1.log 2>&1 || { echo T1FAIL; tail -30 $O/t1.log; exit 1; }
tail -2 $O/t1.log
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_deterministic_gpu.py -k "affine_grid" > $O/t2.log 2>&1 || { echo T2FAIL; tail -30 $O/t2.log; exit 1; }
tail -2 $O/t2.log
for rep in 1 2; do for f in 4 45 46 47; do
  SG2_C64_RING=$f timeout -k 10 120 python -u tools/ring_ab.py 3 >> $O/ring_ab.log 2>&1 || { echo RABFAIL; tail -20 $O/ring_ab.log; exit 1; }
done; done
grep -v amdgpu $O/ring_ab.log
for f in 4 47; do
SG2_C64_RING=$f SG2HIP_LIB=tools/diag_libs/libsg2hip_r512.so timeout -k 10 120 python -u tools/ring_stamps.py > $O/stamps_$f.log 2>&1 || { echo STFAIL; tail -20 $O/stamps_$f.log; exit 1; }
grep -v amdgpu $O/stamps_$f.log
done
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo BFAIL; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-700
