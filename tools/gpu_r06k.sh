#!/bin/bash
# round 6, call k: layer_bwd in-launch deterministic combine -- tests, micro timing, bench
set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_deterministic_gpu.py \
    tests/test_ops_gpu.py tests/test_config_gpu.py -k "det or layer_bwd or fused_synthesis or c2 or c4" > $O/tests.log 2>&1 || { echo TFAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for f in 0 2; do SG2_LB_FORM=$f timeout -k 10 120 python -u tools/lb_micro.py 2>&1 | grep -v amdgpu.ids | tee -a $O/lb.log | grep "C=64 "; done
for f in 0 2 0 2; do
  SG2_LB_FORM=$f timeout -k 10 300 python -u bench.py --steps 48 --no-cpu-baseline --no-roofline > $O/bench_$f.log 2>&1 || { echo BFAIL; tail -20 $O/bench_$f.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_$f.log') if l.startswith('{')][-1]); print('lbform', '$f', d['value'], d['ms_per_step'])"
done
