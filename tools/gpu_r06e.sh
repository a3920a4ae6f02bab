#!/bin/bash
# round 6, call e: two-level det_sum, gather without per-pixel divisions -- tests, bench A/B, det launch shapes
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_deterministic_gpu.py \
    tests/test_ops_gpu.py -k "det or grid_sample or layer_bwd" > $O/tests.log 2>&1 || { echo TFAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in off on off on; do
  timeout -k 10 300 python -u bench.py --steps 48 --no-cpu-baseline --no-roofline --deterministic $m > $O/bench_det_$m.log 2>&1 || { echo BFAIL $m; tail -20 $O/bench_det_$m.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_det_$m.log') if l.startswith('{')][-1]); print('det', '$m', d['value'], d['ms_per_step'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace -d "$O/prof_on" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-roofline --steps 16 --deterministic on > "$O/prof_bench_on.log" 2>&1 || { echo PFAIL; tail -20 $O/prof_bench_on.log; exit 1; }
t=$(find "$O/prof_on" -name 'run_kernel_trace.csv' | head -1)
python3 tools/trace_kstats.py "$t" 'det_sum|finalize|gather' 25 > $O/det_shapes.txt
rm -f "$t"
cat $O/det_shapes.txt
