#!/bin/bash
# A/B builds of conv3x3.hip with compile-time variants (-D flags), timed by conv_micro.py on the 256^2
# C = 64 layer.  Outputs of every variant are correct (unlike c64p_diag.sh's timing-only builds).
#   VARS="SG2_C64P_SST=10 SG2_C64P_SST=7" bash tools/c64p_var.sh build     (CPU)
#   VARS="..." bash tools/c64p_var.sh run                                   (GPU)
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/gan-track_amd/csrc
O=$R/tools/diag_libs
if [ "$1" = build ]; then
    mkdir -p "$O/obj"
    for v in $VARS; do
        t=$(echo "$v" | tr '=,' '__')
        hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $(echo "$v" | tr ',' '\n' | sed 's/^/-D/') -c "$C/conv3x3.hip" -o "$O/obj/conv3x3_$t.o" || exit 1
        objs=$(ls "$C"/build/*.o | grep -v conv3x3.o)
        hipcc -shared --offload-arch=gfx950 -o "$O/libsg2hip_$t.so" $objs "$O/obj/conv3x3_$t.o" || exit 1
    done
else
    cd "$R" || exit 1
    for rep in 1 2; do
        for v in $VARS; do
            t=$(echo "$v" | tr '=,' '__')
            m=$(SG2HIP_LIB=$O/libsg2hip_$t.so timeout -k 10 120 python -u tools/conv_micro.py --which halo --shapes ${SHAPES:-256x64} 2>&1) || exit 1
            r=$(SG2HIP_LIB=$O/libsg2hip_$t.so timeout -k 10 120 python -u tools/roofline_only.py 2>&1) || exit 1
            echo "$t: $(echo "$m" | grep -v amdgpu) || roofline $(echo "$r" | grep -o "'ms_per_launch': [0-9.]*" | head -2 | tr '\n' ' ')"
        done
    done
fi
