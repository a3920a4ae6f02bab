#!/bin/bash
# round 5, call d: ring form 49 (dynamic tail) parity, A/B, stamps
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "c64_ring and 49" > $O/t1.log 2>&1 || { echo T1FAIL; tail -30 $O/t1.log; exit 1; }
tail -1 $O/t1.log
for rep in 1 2; do for f in 46 49; do
  SG2_C64_RING=$f timeout -k 10 120 python -u tools/ring_ab.py 3 2>&1 | grep -v amdgpu | head -1 >> $O/ring_ab.log || { echo RABFAIL; exit 1; }
done; for d in 10 30; do
  SG2_RING_DYN=$d SG2_C64_RING=49 timeout -k 10 120 python -u tools/ring_ab.py 3 2>&1 | grep -v amdgpu | head -1 | sed "s/^/dyn$d /" >> $O/ring_ab.log || { echo RABFAIL; exit 1; }
done; done
cat $O/ring_ab.log
SG2_C64_RING=49 SG2HIP_LIB=tools/diag_libs/libsg2hip_r512.so timeout -k 10 120 python -u tools/ring_stamps.py > $O/stamps_49.log 2>&1 || { echo STFAIL; tail -20 $O/stamps_49.log; exit 1; }
grep -v amdgpu $O/stamps_49.log
