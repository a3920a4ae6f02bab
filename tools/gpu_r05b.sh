#!/bin/bash
# round 5, call b: in-kernel clock of the ring kernel (stamps diag), full vs compute skeleton
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
export PYTHONUNBUFFERED=1
for cfg in "512 4" "512 46" "560 4"; do set -- $cfg
  SG2_C64_RING=$2 SG2HIP_LIB=tools/diag_libs/libsg2hip_r$1.so timeout -k 10 120 python -u tools/ring_stamps.py > $O/stamps_$1_$2.log 2>&1 || { echo STFAIL; tail -20 $O/stamps_$1_$2.log; exit 1; }
  echo "== lib r$1 form $2"; grep -v amdgpu $O/stamps_$1_$2.log
done
