#!/bin/bash
# Timing-only builds of libsg2hip.so for the persistent C=64 conv (SG2_DIAG bits in csrc/conv3x3.hip):
# each removes one part of the kernel so conv_micro.py's times show what that part costs.  Outputs are
# wrong in these builds; they are loaded only through SG2HIP_LIB by the micro-benchmark.
#   bash tools/c64p_diag.sh build        (CPU: compiles tools/diag_libs/libsg2hip_d<bits>.so)
#   bash tools/c64p_diag.sh run          (GPU: conv_micro halo timings per build)
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/gan-track_amd/csrc
O=$R/tools/diag_libs
BITS="${BITS:-2 4 6 8 10}"
if [ "$1" = build ]; then
    mkdir -p "$O/obj"
    for b in $BITS; do
        hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DSG2_DIAG=$b -c "$C/conv3x3.hip" -o "$O/obj/conv3x3_d$b.o" || exit 1
        objs=$(ls "$C"/build/*.o | grep -v conv3x3.o)
        hipcc -shared --offload-arch=gfx950 -o "$O/libsg2hip_d$b.so" $objs "$O/obj/conv3x3_d$b.o" || exit 1
    done
else
    cd "$R" || exit 1
    echo "base: $(timeout -k 10 120 python -u tools/conv_micro.py --which halo --shapes 256x64 2>&1 | grep -v amdgpu)"
    for b in $BITS; do
        echo "d$b: $(SG2HIP_LIB=$O/libsg2hip_d$b.so timeout -k 10 120 python -u tools/conv_micro.py --which halo --shapes 256x64 2>&1 | grep -v amdgpu)" || exit 1
    done
fi
