#!/bin/bash
# round 6, call au: small-batch FC kernels (sg2_fc_gemm / sg2_fc_wgrad) -- parity, glue time, bench A/B
set -o pipefail
O=gpurun_out/r06au
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_capi.py tests/test_ops_gpu.py -k "capi or fc_kernels or mapping or grouped or torgb" > $O/tests.log 2>&1 || { echo TFAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_train_gpu.py tests/test_trainer_gpu.py tests/test_bench_gpu.py > $O/tests2.log 2>&1 || { echo T2FAIL; tail -40 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
timeout -k 10 300 python -u tools/glue_time.py 4 > $O/glue_time.txt 2>&1 || { echo GFAIL; tail -20 $O/glue_time.txt; exit 1; }
grep -E "torch kernels|addmm|aten::mm" $O/glue_time.txt | head -8
for t in 1 0 1 0; do
SG2_FC=$t timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $O/bench_$t.log 2>&1 || { echo BFAIL; tail -20 $O/bench_$t.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_$t.log') if l.startswith('{')][-1]); print('fc', $t, d['value'], d['ms_per_step'])"
done
