#!/bin/bash
# round 6, call c: deterministic-mode kernels (slots, fused finalize, one-launch det_sum) -- tests, bench A/B, profile
set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_deterministic_gpu.py \
    tests/test_ops_gpu.py -k "det or conv3x3 or grid_sample or c64 or ring or layer_bwd or wgrad or split" > $O/tests.log 2>&1 || { echo TFAIL; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for m in off on off on; do
  timeout -k 10 300 python -u bench.py --steps 48 --no-cpu-baseline --no-roofline --deterministic $m > $O/bench_det_$m.log 2>&1 || { echo BFAIL $m; tail -20 $O/bench_det_$m.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_det_$m.log') if l.startswith('{')][-1]); print('det', '$m', d['value'], d['ms_per_step'])"
done
for m in off on; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_$m" -o run --output-format csv \
      -- python3 "$R/bench.py" --no-cpu-baseline --no-roofline --steps 16 --deterministic $m > "$O/prof_bench_$m.log" 2>&1 || { echo PFAIL $m; tail -20 $O/prof_bench_$m.log; exit 1; }
  find "$O/prof_$m" -name 'run_kernel_trace.csv' -delete
done
python3 tools/kdiff.py $(find $O/prof_off -name run_kernel_stats.csv) $(find $O/prof_on -name run_kernel_stats.csv) 30 > $O/kdiff.txt
cat $O/kdiff.txt
