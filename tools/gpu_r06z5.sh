#!/bin/bash
# round 6, call z5: deterministic grid-sample gather with the tight scan box -- parity, timing in the step
set -o pipefail
O=gpurun_out/r06z5
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_deterministic_gpu.py tests/test_ops_gpu.py \
    -k "grid_sample or augment or gather or dynamic" > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_bench_gpu.py > $O/tb.log 2>&1 || { echo BTFAIL; tail -30 $O/tb.log; exit 1; }
tail -1 $O/tb.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o b -- python3 bench.py --steps 32 --no-cpu-baseline --no-roofline > $O/bprof.log 2>&1 || { echo PFAIL; tail -20 $O/bprof.log; exit 1; }
grep -h "grid_sample\|zero_region\|upfirdn_1d" $O/prof/*stats.csv | cut -c1-200 | head -12
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$i.log 2>&1 || { echo BFAIL; tail -20 $O/bench_$i.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
