#!/bin/bash
# round 6, call aw: parameter-layout slot sum with an LDS transpose -- parity, kernel time, bench
set -o pipefail
O=gpurun_out/r06aw
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_capi.py tests/test_ops_gpu.py tests/test_deterministic_gpu.py -k "capi or wgrad or det or fused or torgb or synthesis or layer or up or vjp or double" > $O/tests.log 2>&1 || { echo TFAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_train_gpu.py tests/test_trainer_gpu.py tests/test_bench_gpu.py > $O/tests2.log 2>&1 || { echo T2FAIL; tail -40 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 16 --no-cpu-baseline --no-roofline > $O/prof.log 2>&1 || { echo PFAIL; tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name 'run_kernel_stats.csv' | head -1); grep -h "det_sum" "$f" | cut -c1-160
find $O/prof -name 'run_kernel_trace.csv' -delete
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$i.log 2>&1 || { echo BFAIL; tail -20 $O/bench_$i.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
