#!/bin/bash
# round 6, call m: split targets under the deterministic default (env knobs, read once per process), same box
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {
  env "$@" timeout -k 10 300 python -u bench.py --steps 48 --no-cpu-baseline --no-roofline > $O/b.log 2>&1 || { echo BFAIL "$@"; tail -20 $O/b.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1]); print('$*', d['value'], d['ms_per_step'])" | tee -a $O/sweep.txt
}
run X=base
run SG2_CONV_SPLIT_WGS=256
run SG2_CONV_SPLIT_WGS=1024
run X=base
run SG2_CWGRAD_WGS=1024
run SG2_CWGRAD_WGS=512
run SG2_CWGRAD_WGS=4096
run X=base
run SG2_WGRAD_WGS=192
run SG2_WGRAD_WGS=384
run X=base
