#!/bin/bash
# A/B of the generic weight-gradient kernel (f32 split form): tools/_old/libsg2hip.so vs the in-tree build.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-wgab}
mkdir -p "$O"
cd "$R" || exit 1
for v in new old new; do
    if [ $v = old ]; then export SG2HIP_LIB=$R/tools/_old/libsg2hip.so; else unset SG2HIP_LIB; fi
    echo "== $v"
    timeout -k 10 120 python -u tools/conv_micro.py --dtype float32 --which wgrad --shapes 16x512,8x512 \
        > "$O/$v.log" 2>&1 || exit $?
    grep -v amdgpu.ids "$O/$v.log"
done
