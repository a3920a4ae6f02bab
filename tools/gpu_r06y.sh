#!/bin/bash
# round 6, call y: glue census; det_sum call shapes with their dispatch times
set -o pipefail
O=gpurun_out/r06y
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u tools/glue_census.py > $O/glue.txt 2>&1 || { echo GFAIL; tail -20 $O/glue.txt; exit 1; }
SG2_DET_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o det -- python3 tools/det_trace.py 2> $O/calls.txt > $O/det_trace.log || { echo DFAIL; tail -20 $O/calls.txt; exit 1; }
ls -R $O/prof | head
