#!/bin/bash
# round 6, call b: kernel-trace stats of the bench with the deterministic mode off / on (where the det cost goes)
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$(pwd)
for m in off on; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_$m" -o run --output-format csv \
      -- python3 "$R/bench.py" --no-cpu-baseline --no-roofline --steps 16 --deterministic $m > "$O/prof_bench_$m.log" 2>&1 || { echo PFAIL $m; tail -20 $O/prof_bench_$m.log; exit 1; }
  find "$O/prof_$m" -name 'run_kernel_trace.csv' -delete
done
python3 tools/kdiff.py $(find $O/prof_off -name run_kernel_stats.csv) $(find $O/prof_on -name run_kernel_stats.csv) 40 > $O/kdiff.txt
cat $O/kdiff.txt
