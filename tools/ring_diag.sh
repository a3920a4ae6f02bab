#!/bin/bash
# Timing-only builds of the ring C=64 conv (SG2_RDIAG bits in csrc/conv3x3.hip: 16 no loads, 32 no stores, 64 no
# MFMA); outputs are wrong in these builds, which only tools/ring_ab.py loads through SG2HIP_LIB.
#   bash tools/ring_diag.sh build   (CPU)        bash tools/ring_diag.sh run   (GPU)
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/gan-track_amd/csrc
O=$R/tools/diag_libs
BITS="${BITS:-16 32 48 64 80 96}"
if [ "$1" = build ]; then
    mkdir -p "$O/obj"
    for b in $BITS; do
        hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DSG2_RDIAG=$b -c "$C/conv3x3.hip" -o "$O/obj/conv3x3_r$b.o" &
    done
    wait
    for b in $BITS; do
        objs=$(ls "$C"/build/*.o | grep -v conv3x3.o)
        hipcc -shared --offload-arch=gfx950 -o "$O/libsg2hip_r$b.so" $objs "$O/obj/conv3x3_r$b.o" || exit 1
    done
else
    cd "$R" || exit 1
    for rep in 1 2; do
        timeout -k 10 120 python -u tools/ring_ab.py 3 2>&1 | grep -v amdgpu || exit 1
        for b in $BITS; do
            echo "r$b: $(SG2HIP_LIB=$O/libsg2hip_r$b.so timeout -k 10 120 python -u tools/ring_ab.py 3 2>&1 | grep -v amdgpu | head -1)" || exit 1
        done
    done
fi
