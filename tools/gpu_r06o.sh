#!/bin/bash
# round 6, call o: grid-sample kernels with 32-bit index math -- tests and timing
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_deterministic_gpu.py \
    tests/test_ops_gpu.py -k "grid_sample or augment or no_dynamic_tail" > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u tools/gs_micro.py 2>&1 | grep -v amdgpu.ids | tee $O/gs.txt
SG2HIP_LIB=$(pwd)/tools/diag_libs/lib_before.so timeout -k 10 120 python -u tools/gs_micro.py 2>&1 | grep -v amdgpu.ids | sed 's/^/before: /' | tee -a $O/gs.txt
