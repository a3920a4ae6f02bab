#!/bin/bash
# usage: tools/gpurun_bg.sh <delay-seconds> '<remote command>'   (one gpurun call; logs under gpurun_out/)
sleep "$1"
cd /root/repo && make -s -C gan-track_amd/csrc -j8 || exit 1
rm -f gpurun_out/*.log
timeout 1500 /usr/local/graft/bin/gpurun --timeout 900 -- "$2" > gpurun_out/call.txt 2>&1
tail -3 gpurun_out/call.txt
