#!/bin/bash
# A/B of the FIR kernels: tools/_old/libsg2hip.so vs the in-tree build (tools/fir_micro.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-firab}
mkdir -p "$O"
cd "$R" || exit 1
for v in new old; do
    if [ $v = old ]; then export SG2HIP_LIB=$R/tools/_old/libsg2hip.so; else unset SG2HIP_LIB; fi
    echo "== $v"
    timeout -k 10 120 python -u tools/fir_micro.py > "$O/$v.log" 2>&1 || exit $?
    grep -v amdgpu.ids "$O/$v.log"
done
