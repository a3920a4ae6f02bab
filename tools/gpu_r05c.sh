#!/bin/bash
# round 5, call c: ring form 48 parity, A/B of 4 / 46 / 48, stamps with tail statistics
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "c64_ring and 48" > $O/t1.log 2>&1 || { echo T1FAIL; tail -30 $O/t1.log; exit 1; }
tail -1 $O/t1.log
for rep in 1 2; do for f in 4 46 48; do
  SG2_C64_RING=$f timeout -k 10 120 python -u tools/ring_ab.py 3 2>&1 | grep -v amdgpu | head -1 >> $O/ring_ab.log || { echo RABFAIL; exit 1; }
done; done
cat $O/ring_ab.log
for f in 46 48; do
  SG2_C64_RING=$f SG2HIP_LIB=tools/diag_libs/libsg2hip_r512.so timeout -k 10 120 python -u tools/ring_stamps.py > $O/stamps_$f.log 2>&1 || { echo STFAIL; tail -20 $O/stamps_$f.log; exit 1; }
  echo "== form $f"; grep -v amdgpu $O/stamps_$f.log
done
