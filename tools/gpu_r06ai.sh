#!/bin/bash
# round 6, call ai: reflect pad over its read region only -- parity, det ADA micro, bench-step tests, bench
set -o pipefail
O=gpurun_out/r06ai
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_deterministic_gpu.py \
    -k "upfirdn or augment or dynamic or gather or reflect or grid_sample" > $O/tests.log 2>&1 || { echo TFAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/ada_micro.py 40 det > $O/ada_det.txt 2>&1 || { echo AFAIL; tail -20 $O/ada_det.txt; exit 1; }
grep -E "ADA|reflect" $O/ada_det.txt
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_bench_gpu.py > $O/tb.log 2>&1 || { echo BTFAIL; tail -30 $O/tb.log; exit 1; }
tail -1 $O/tb.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$i.log 2>&1 || { echo BFAIL; tail -20 $O/bench_$i.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
