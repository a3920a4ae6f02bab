#!/bin/bash
# round 6, call af: SQ counters of the 1-D FIR vertical pass (ADA micro) and the 4x4 FIR strip kernel (FIR micro)
set -o pipefail
O=gpurun_out/r06af
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
ADA_NOPROF=1 bash tools/pmc_kernel.sh $O/vrun 'upfirdn_1d_vrun' tools/ada_micro.py 4 det > $O/vrun.txt 2>&1 || { echo V; tail -20 $O/vrun.txt; exit 1; }
bash tools/pmc_kernel.sh $O/f4s 'upfirdn_nhwc_f4s' tools/fir_micro.py > $O/f4s.txt 2>&1 || { echo F; tail -20 $O/f4s.txt; exit 1; }
cat $O/vrun.txt | tail -30
cat $O/f4s.txt | tail -30
rm -rf $O/vrun/p* $O/f4s/p*
