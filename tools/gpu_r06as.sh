#!/bin/bash
# round 6, call as: f32 weight gradients in the parameter layout (sg2_conv2d_wgrad_oikk) -- parity, glue time, bench
set -o pipefail
O=gpurun_out/r06as
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_capi.py tests/test_ops_gpu.py tests/test_deterministic_gpu.py -k "capi or wgrad or det or fused or torgb or synthesis or layer or up or vjp or double" > $O/tests.log 2>&1 || { echo TFAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_train_gpu.py tests/test_trainer_gpu.py tests/test_bench_gpu.py > $O/tests2.log 2>&1 || { echo T2FAIL; tail -40 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
timeout -k 10 300 python -u tools/glue_time.py 4 > $O/glue_time.txt 2>&1 || { echo GFAIL; tail -20 $O/glue_time.txt; exit 1; }
grep -E "torch kernels|512, 512, 3, 3" $O/glue_time.txt | head -6
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$i.log 2>&1 || { echo BFAIL; tail -20 $O/bench_$i.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_$i.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
