#!/bin/bash
# round 5, call ab: C1 same-state 16-bit parity; up-2 edge split (the last cell row / column as three-tap strips): tests, A/B, step A/B
set -o pipefail
O=gpurun_out/r05ab
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "up2" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_config_gpu.py -k "16bit and c1" > $O/c1_16.log 2>&1 || { tail -40 $O/c1_16.log; exit 1; }
tail -2 $O/c1_16.log
timeout -k 10 180 python -u tools/up2_ab.py > $O/up2_ab.log 2>&1 || { tail -20 $O/up2_ab.log; exit 1; }
cat $O/up2_ab.log
for m in 64 16; do
  SG2_UP2_MIN=$m timeout -k 10 300 python -u bench.py > $O/bench_min$m.log 2>&1 || { tail -20 $O/bench_min$m.log; exit 1; }
  echo "min=$m $(grep -o '"value": [0-9.]*, "unit": "[^"]*", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' $O/bench_min$m.log)"
done
