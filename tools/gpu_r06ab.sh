#!/bin/bash
# round 6, call ab: det_sum vectorised small-S form and multi-job launches (layer_bwd) -- det tests, bench x2
set -o pipefail
O=gpurun_out/r06ab
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_deterministic_gpu.py tests/test_bench_gpu.py > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "layer or wgrad or det or dot" > $O/tests2.log 2>&1 || { echo T2FAIL; tail -30 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$i.log 2>&1 || { echo BFAIL; tail -20 $O/bench_$i.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
