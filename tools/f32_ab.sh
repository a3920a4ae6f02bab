#!/bin/bash
# A/B of the f32 (split-bf16) conv kernels: tools/_old/libsg2hip.so vs the in-tree build.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-f32ab}
mkdir -p "$O"
cd "$R" || exit 1
for v in new old; do
    if [ $v = old ]; then export SG2HIP_LIB=$R/tools/_old/libsg2hip.so; else unset SG2HIP_LIB; fi
    echo "== $v"
    timeout -k 10 120 python -u tools/conv_micro.py --dtype float32 --which generic --shapes 16x512 \
        > "$O/$v.log" 2>&1 || exit $?
    timeout -k 10 120 python -u tools/conv_micro.py --dtype float16 --which halo \
        >> "$O/$v.log" 2>&1 || exit $?
    grep -v amdgpu.ids "$O/$v.log"
done
